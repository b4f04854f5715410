#!/bin/bash
# Round 3: deferred-count DP step at world 2 with an overflowing rank, step end event -- new tests first, whole GPU
# suite, step timeline, bench, prefilter / scan LDS PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_w}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dp.py tests/test_post_bulk.py > $OUT/pytest_first.log 2>&1 && echo FIRST_OK || { tail -40 $OUT/pytest_first.log; exit 1; }
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
