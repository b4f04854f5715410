#!/bin/bash
# Ingest probe (SDMA vs pull kernel, NUMA binding) + headline bench + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 200 python tools/h2d_probe.py > gpurun_out/h2d.log 2>&1 && echo PROBE_OK &&
timeout -k 10 200 python tools/h2d_probe.py --bind > gpurun_out/h2d_bind.log 2>&1 && echo PROBE_BIND_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --profile > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/rocprof.log 2>&1 && echo ROCPROF_OK
