#!/bin/bash
# Round 3: fused DFA+BPG candidate verify (request path) -- GPU tests, request trace; bulk step timelines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_r}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bpg.py tests/test_gpu.py tests/test_gpu_serving.py > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/req -o run -- python3 $R/tools/request_trace.py --requests 300 > $R/$OUT/req.log 2>&1 && echo REQ_OK || { tail -20 $R/$OUT/req.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk_noov -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/bulk_noov.log 2>&1 && echo BULK_NOOV_OK || { tail -20 $R/$OUT/bulk_noov.log; exit 1; }
cd $R
python tools/request_trace.py --db $(ls $OUT/req/*/run_results.db $OUT/req/run_results.db 2>/dev/null | head -1) --requests 300 > $OUT/req_kernels.txt 2>&1 || true
head -8 $OUT/req_kernels.txt; grep p50 $OUT/req.log | tail -1
for v in bulk bulk_noov; do
  DB=$(ls $OUT/$v/*/run_results.db $OUT/$v/run_results.db 2>/dev/null | head -1)
  python tools/step_timeline.py $DB --skip 3 > $OUT/timeline_$v.txt 2>&1 || true
  python tools/kstats_db.py $DB 4 60 --median --marker k_nl_count --last 4 > $OUT/kernels_$v.txt 2>&1 || true
  head -2 $OUT/timeline_$v.txt; tail -1 $OUT/kernels_$v.txt
done
rm -rf $OUT/req $OUT/bulk $OUT/bulk_noov
