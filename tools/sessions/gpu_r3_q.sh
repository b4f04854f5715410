#!/bin/bash
# Round 3: bulk step timeline (kernel durations + host gaps) on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk_noov -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/bulk_noov.log 2>&1 && echo BULK_NOOV_OK || { tail -20 $R/$OUT/bulk_noov.log; exit 1; }
cd $R
for v in bulk bulk_noov; do
  DB=$(ls $OUT/$v/*/run_results.db $OUT/$v/run_results.db 2>/dev/null | head -1)
  python tools/step_timeline.py $DB --skip 3 > $OUT/timeline_$v.txt 2>&1 || true
  python tools/kstats_db.py $DB 4 60 --median --marker k_nl_count --last 4 > $OUT/kernels_$v.txt 2>&1 || true
  head -3 $OUT/timeline_$v.txt; tail -1 $OUT/kernels_$v.txt
done
rm -rf $OUT/bulk $OUT/bulk_noov
