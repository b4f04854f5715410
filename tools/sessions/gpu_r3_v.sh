#!/bin/bash
# Round 3: deferred-count DP step (no mid-step read) -- new tests first, whole GPU
# suite, step timeline, bench, prefilter / scan LDS PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_v}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_post_bulk.py tests/test_gpu.py tests/test_dp.py tests/test_bench.py > $OUT/pytest_first.log 2>&1 && echo FIRST_OK || { tail -40 $OUT/pytest_first.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk_noov -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/bulk_noov.log 2>&1 && echo BULK_NOOV_OK || { tail -20 $R/$OUT/bulk_noov.log; exit 1; }
cd $R
DB=$(ls $OUT/bulk_noov/*/run_results.db $OUT/bulk_noov/run_results.db 2>/dev/null | head -1)
python tools/step_timeline.py $DB --skip 3 > $OUT/timeline_bulk_noov.txt 2>&1 || true
head -14 $OUT/timeline_bulk_noov.txt
rm -rf $OUT/bulk_noov
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'],d['matcher_counts_rank0'])"
cd /tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_prefilter|k_scan_multi" --output-format csv -d $R/$OUT/pmc/p1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --parse-requests 0 --backend none > $R/$OUT/pmc_1.log 2>&1 || { echo "PMC failed"; tail -5 $R/$OUT/pmc_1.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_bulk.md 2>&1 || true
cut -c1-400 $OUT/pmc_bulk.md
rm -rf $OUT/pmc
