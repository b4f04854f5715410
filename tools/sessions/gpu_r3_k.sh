#!/bin/bash
# Round 3: wave load-balanced k_pf_verify + trimmed cooperative BPG walk -- GPU tests (BPG under every
# walk mode, prefilter / engine suites), request trace and bulk kernel table, A/B against the old kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_k}
mkdir -p $OUT
for w in auto coop; do
  LP_BPG_WALK=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bpg.py > $OUT/pytest_bpg_$w.log 2>&1 && echo BPG_TESTS_${w}_OK || { tail -40 $OUT/pytest_bpg_$w.log; exit 1; }
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_prefilter_tables.py tests/test_post.py tests/test_pipeline.py > $OUT/pytest_core.log 2>&1 && echo CORE_TESTS_OK || { tail -40 $OUT/pytest_core.log; exit 1; }
tail -1 $OUT/pytest_core.log
cd /tmp && export TMPDIR=/tmp
run_req() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/req_$name -o run -- python3 $R/tools/request_trace.py --requests 300 > $R/$OUT/req_$name.log 2>&1 && echo REQ_${name}_OK || { tail -20 $R/$OUT/req_$name.log; return 1; }
}
run_bulk() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk_$name -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk_$name.log 2>&1 && echo BULK_${name}_OK || { tail -20 $R/$OUT/bulk_$name.log; return 1; }
}
run_req new LP_X=0 && run_req old LP_BPG_WALK=lane LP_PF_VERIFY=lanes && run_bulk new LP_X=0 && run_bulk old LP_PF_VERIFY=lanes || exit 1
cd $R
for w in new old; do
  python tools/request_trace.py --db $(ls $OUT/req_$w/*/run_results.db $OUT/req_$w/run_results.db 2>/dev/null | head -1) --requests 300 > $OUT/req_kernels_$w.txt 2>&1 || true
  head -6 $OUT/req_kernels_$w.txt; grep p50 $OUT/req_$w.log | tail -1
  python tools/kstats_db.py $(ls $OUT/bulk_$w/*/run_results.db $OUT/bulk_$w/run_results.db 2>/dev/null | head -1) 7 45 --median > $OUT/bulk_kernels_$w.txt 2>&1 || true
  grep -i "verify\|bpg\|total" $OUT/bulk_kernels_$w.txt; tail -1 $OUT/bulk_$w.log | cut -c1-300
done
rm -rf $OUT/req_new $OUT/req_old $OUT/bulk_new $OUT/bulk_old
