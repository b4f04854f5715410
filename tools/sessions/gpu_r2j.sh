#!/bin/bash
# Round-2: two-pass line index (count / scan / lines), one-read matcher arena, packed events.
set -o pipefail
OUT=${OUT:-gpurun_out/r2j}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_summarize.py > $OUT/pytest_a.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 8 --warmup 2 --parse-requests 0 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/req -o req -- python tools/request_trace.py --requests 200 > $OUT/request_trace.json 2> $OUT/request_trace.err || exit 1
