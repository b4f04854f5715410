#!/bin/bash
# headline bench (overlapped + serial + per-stage) + rocprofv3 kernel stats + single config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-overlap > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err && echo SERIAL_OK &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --profile > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > gpurun_out/cfg_single.json 2> gpurun_out/cfg_single.err && echo SINGLE_OK &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/rocprof.log 2>&1 && echo ROCPROF_OK
