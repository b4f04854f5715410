#!/bin/bash
# Round 3: k_feat_cov lines per workgroup A/B (LP_FC_PER) -- kernel tables of the bulk step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_af}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for per in 4096 1024 256; do
  LP_FC_PER=$per timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$per -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$per.log 2>&1 && echo TL_${per}_OK || { tail -20 $R/$OUT/tl_$per.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$per/*/run_results.db $R/$OUT/tl_$per/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $R/$OUT/bulk_kernels_fc$per.txt 2>&1 || true
  grep "k_feat_cov\|k_nl_count" $R/$OUT/bulk_kernels_fc$per.txt
  rm -rf $R/$OUT/tl_$per
done
