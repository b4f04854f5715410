#!/bin/bash
# k_fetch inputs A/B + NUMA-bound server: GPU tests, engine p50 (fetch on / off / on), request
# trace with k_fetch, /parse breakdown, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2q}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
T="timeout -k 10 200 python tools/request_trace.py --requests 400"
$T > $OUT/ab.jsonl 2>/dev/null && echo fetch_ok || exit 1
LP_RUNNER_FETCH=0 $T >> $OUT/ab.jsonl 2>/dev/null && echo sdma_ok || exit 1
$T >> $OUT/ab.jsonl 2>/dev/null && echo fetch2_ok || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RT_OK || exit 1
cd $R
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
rm -rf $OUT/req
timeout -k 10 200 python tools/parse_breakdown.py --n 300 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
