#!/bin/bash
# Round 3: k_feat_cov phase probe (LP_FC_PROBE: 0 = normal, 1 = no walks, 2 = per-line loads only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_al}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for pr in 0 1 2; do
  LP_FC_PROBE=$pr timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$pr -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$pr.log 2>&1 && echo TL_${pr}_OK || { tail -20 $R/$OUT/tl_$pr.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$pr/*/run_results.db $R/$OUT/tl_$pr/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $R/$OUT/bulk_kernels_probe$pr.txt 2>&1 || true
  grep "k_feat_cov" $R/$OUT/bulk_kernels_probe$pr.txt
  rm -rf $R/$OUT/tl_$pr
done
