#!/bin/bash
# Round 3: A/B -- does k_pf_verify overlap k_scan_multi when launched first with a small grid?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_y}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in "0 8192" "1 256" "1 1024" "1 8192"; do
  set -- $cfg
  tag=first$1_grid$2
  LP_PFV_FIRST=$1 LP_PFV_GRID=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$tag -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$tag.log 2>&1 && echo TL_${tag}_OK || { tail -20 $R/$OUT/tl_$tag.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$tag/*/run_results.db $R/$OUT/tl_$tag/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 > $R/$OUT/timeline_$tag.txt 2>&1 || true
  head -1 $R/$OUT/timeline_$tag.txt
  grep -E "k_scan_multi|k_pf_verify|k_prefilter" $R/$OUT/timeline_$tag.txt | head -3
  rm -rf $R/$OUT/tl_$tag
done
