#!/bin/bash
# Round 3 final-tree check (after the row-offset context walk): smoke, whole GPU suite, driver-style bench, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_final2}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 > $R/$OUT/rocprof.log 2>&1 && echo ROCPROF_OK || { tail -20 $R/$OUT/rocprof.log; exit 1; }
cd $R
STATS=$(ls $OUT/prof/*/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -1)
cp "$STATS" $OUT/kernel_stats.csv 2>/dev/null || true
DB=$(ls $OUT/prof/*/run_results.db $OUT/prof/run_results.db 2>/dev/null | head -1)
python3 tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $OUT/bulk_kernels.txt 2>&1 || true
head -30 $OUT/bulk_kernels.txt
rm -rf $OUT/prof
