#!/bin/bash
# prefilter experiments: GPU tests, profiled bench (stage timings), rocprof kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu1.log 2>&1 && echo T_OK &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/bench.json 2>/dev/null && echo PROF_OK
