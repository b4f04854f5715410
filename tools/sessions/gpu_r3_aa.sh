#!/bin/bash
# Round 3: A/B of the bulk BPG verify walk (one lane per key vs 16-lane cooperative) and of the
# literal verify's lanes per filter hit (4 / 8 / 16), on the bulk step timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_aa}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_post_bulk.py tests/test_gpu.py > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
LP_BPG_WALK=coop LP_PFV_LANES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_post_bulk.py tests/test_gpu.py tests/test_bpg.py > $OUT/pytest_ab.log 2>&1 && echo AB_TESTS_OK || { tail -40 $OUT/pytest_ab.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for cfg in "auto 4" "coop 4" "auto 8" "auto 16"; do
  set -- $cfg
  tag=walk$1_lanes$2
  LP_BPG_WALK=$1 LP_PFV_LANES=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$tag -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$tag.log 2>&1 && echo TL_${tag}_OK || { tail -20 $R/$OUT/tl_$tag.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$tag/*/run_results.db $R/$OUT/tl_$tag/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 > $R/$OUT/timeline_$tag.txt 2>&1 || true
  head -1 $R/$OUT/timeline_$tag.txt
  grep -E "k_pf_verify|bpg|k_scan_multi|k_summ" $R/$OUT/timeline_$tag.txt | head -6
  rm -rf $R/$OUT/tl_$tag
done
