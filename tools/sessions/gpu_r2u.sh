#!/bin/bash
# Bulk scan 64-byte superblocks A/B (LP_SCAN_SB64=1 / 0) + scan GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2u}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan_multi.py tests/test_gpu.py > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  LP_SCAN_SB64=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/p$v -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 > $R/$OUT/bench_sb$v.json 2> $R/$OUT/bench_sb$v.err && echo SB${v}_OK || exit 1
  (cd $R && python tools/kstats_db.py $OUT/p$v/run_results.db 8 12 --median > $OUT/kernel_table_sb$v.txt 2>&1; rm -rf $OUT/p$v)
done
