#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-overlap > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err && echo BENCH_SERIAL_OK &&
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/rocprof.log 2>&1) && echo ROCPROF_OK &&
bash tools/gpu_pmc.sh
