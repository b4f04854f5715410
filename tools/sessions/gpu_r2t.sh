#!/bin/bash
# Bulk scan A/B: LP_SCAN_VARIANT 0 (inline re-walk) / 1 (queued, 8 waves/SIMD) / 2 (queued, 1 block per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2t}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2; do
  LP_SCAN_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/p$v -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 > $R/$OUT/bench_v$v.json 2> $R/$OUT/bench_v$v.err && echo V${v}_OK || exit 1
  (cd $R && python tools/kstats_db.py $OUT/p$v/run_results.db 8 12 --median > $OUT/kernel_table_v$v.txt 2>&1; rm -rf $OUT/p$v)
done
