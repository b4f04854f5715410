#!/bin/bash
# quick GPU check: pytest -m gpu, profiled bench (mfma vs dfa context engine), rocprof stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
LINES=${LINES:-12500000}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --profile --lines-per-gpu $LINES > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
ENGINE_CONTEXT_ENGINE=dfa timeout -k 10 400 python bench.py --steps 5 --warmup 2 --profile --lines-per-gpu $LINES > gpurun_out/bench_profile_dfa.json 2> gpurun_out/bench_profile_dfa.err && echo PROFILE_DFA_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --lines-per-gpu $LINES > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --lines-per-gpu $LINES > $R/gpurun_out/rocprof.log 2>&1 && echo ROCPROF_OK
