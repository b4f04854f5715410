#!/bin/bash
# RawLogs on the GPU server: GPU tests, /parse breakdown with tail percentiles, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2r}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 200 python tools/parse_breakdown.py --n 400 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --parse-requests 400 > $OUT/bench400.json 2> $OUT/bench400.err && echo BENCH400_OK || exit 1
