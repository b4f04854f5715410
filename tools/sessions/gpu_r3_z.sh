#!/bin/bash
# Round 3: summary chunks of 1024 rows for k <= 256; dual-run scan walk A/B (LP_SCAN_DUAL=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_z}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_summarize.py tests/test_scan_multi.py tests/test_post_bulk.py tests/test_gpu.py tests/test_dp.py > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
LP_SCAN_DUAL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan_multi.py tests/test_post_bulk.py tests/test_gpu.py > $OUT/pytest_dual.log 2>&1 && echo DUAL_TESTS_OK || { tail -40 $OUT/pytest_dual.log; exit 1; }
tail -1 $OUT/pytest_dual.log
cd /tmp && export TMPDIR=/tmp
for dual in 0 1; do
  LP_SCAN_DUAL=$dual timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$dual -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$dual.log 2>&1 && echo TL_${dual}_OK || { tail -20 $R/$OUT/tl_$dual.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$dual/*/run_results.db $R/$OUT/tl_$dual/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 > $R/$OUT/timeline_dual$dual.txt 2>&1 || true
  head -1 $R/$OUT/timeline_dual$dual.txt
  grep -E "k_scan_multi|k_summ_level" $R/$OUT/timeline_dual$dual.txt | head -5
  rm -rf $R/$OUT/tl_$dual
done
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'])"
