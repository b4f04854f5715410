#!/bin/bash
# Round 3: wave-cooperative BPG candidate walk -- kernel tests, request trace (coop vs lane A/B), bulk kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_i}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bpg.py > $OUT/pytest_bpg.log 2>&1 && echo BPG_TESTS_OK || { tail -40 $OUT/pytest_bpg.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for w in coop lane; do
  LP_BPG_WALK=$w timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/req_$w -o run -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/req_$w.log 2>&1 && echo REQ_${w}_OK || { tail -20 $R/$OUT/req_$w.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
cd $R
for w in coop lane; do
  python tools/request_trace.py --db $(ls $OUT/req_$w/*/run_results.db $OUT/req_$w/run_results.db 2>/dev/null | head -1) --requests 200 > $OUT/req_kernels_$w.txt 2>&1 || true
  head -6 $OUT/req_kernels_$w.txt; grep p50 $OUT/req_$w.log | tail -1
done
python tools/kstats_db.py $(ls $OUT/bulk/*/run_results.db $OUT/bulk/run_results.db 2>/dev/null | head -1) 7 45 --median > $OUT/bulk_kernels.txt 2>&1 || true
grep -i bpg $OUT/bulk_kernels.txt; tail -1 $OUT/bulk.log
rm -rf $OUT/req_coop $OUT/req_lane $OUT/bulk
