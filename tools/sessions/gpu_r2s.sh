#!/bin/bash
# Bulk scan with queued hot blocks (8 waves/SIMD) + 2-block look-ahead DFA walks: GPU tests,
# headline bench, bulk kernel stats, request trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
timeout -k 10 200 python tools/request_trace.py --requests 400 > $OUT/rt.json 2>/dev/null && echo RT_OK || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 8 --warmup 2 --parse-requests 0 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err && echo PROF_OK || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RTP_OK || exit 1
cd $R
python tools/kstats_db.py $OUT/prof/run_results.db 10 30 --median > $OUT/kernel_table.txt 2>&1 || true
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
rm -rf $OUT/req
