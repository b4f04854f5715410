#!/bin/bash
# Round 3: short-literal bloom tier on the device -- full GPU suite, kernel table, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_p}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
cd $R
DB=$(ls $OUT/bulk/*/run_results.db $OUT/bulk/run_results.db 2>/dev/null | head -1)
python tools/kstats_db.py $DB 7 60 --median > $OUT/bulk_kernels_all7.txt 2>&1 || true
python tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $OUT/bulk_kernels.txt 2>&1 || true
head -14 $OUT/bulk_kernels_all7.txt; tail -1 $OUT/bulk_kernels.txt
rm -rf $OUT/bulk
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'],d['matcher_counts_rank0'])"
