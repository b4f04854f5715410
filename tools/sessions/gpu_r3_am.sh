#!/bin/bash
# Round 3: context features on row-offset tables (one add + one LDS read per DFA per byte) -- tests, kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_am}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_post_bulk.py tests/test_scan_multi.py > $OUT/pytest_first.log 2>&1 && echo FIRST_OK || { tail -40 $OUT/pytest_first.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl.log 2>&1 && echo TL_OK || { tail -20 $R/$OUT/tl.log; exit 1; }
DB=$(ls $R/$OUT/tl/*/run_results.db $R/$OUT/tl/run_results.db 2>/dev/null | head -1)
python3 $R/tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $R/$OUT/bulk_kernels_noov.txt 2>&1 || true
head -12 $R/$OUT/bulk_kernels_noov.txt
rm -rf $R/$OUT/tl
