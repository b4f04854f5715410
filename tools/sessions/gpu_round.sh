#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench (profiled + headline) -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first failure stops it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-10}
LINES=${LINES:-12500000}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --profile --lines-per-gpu $LINES > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 --lines-per-gpu $LINES > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 --no-overlap --lines-per-gpu $LINES > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err && echo BENCH_SERIAL_OK &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --lines-per-gpu $LINES > $R/gpurun_out/rocprof.log 2>&1 && echo ROCPROF_OK
