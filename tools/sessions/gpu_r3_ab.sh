#!/bin/bash
# Round 3: line index pass 1 folded into the literal prefilter -- new test first, whole GPU suite,
# step timeline (fused vs LP_FUSED_NL=0), bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_ab}
mkdir -p $OUT
LP_FUSED_NL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_post_bulk.py tests/test_dp.py tests/test_bench.py > $OUT/pytest_first.log 2>&1 && echo FIRST_OK || { tail -40 $OUT/pytest_first.log; exit 1; }
LP_FUSED_NL=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  LP_FUSED_NL=$f timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$f -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$f.log 2>&1 && echo TL_${f}_OK || { tail -20 $R/$OUT/tl_$f.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$f/*/run_results.db $R/$OUT/tl_$f/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 --marker k_nl_lines > $R/$OUT/timeline_fused$f.txt 2>&1 || true
  python3 $R/tools/kstats_db.py $DB 5 60 --median --marker k_nl_lines --last 5 > $R/$OUT/bulk_kernels_fused$f.txt 2>&1 || true
  head -12 $R/$OUT/bulk_kernels_fused$f.txt
  rm -rf $R/$OUT/tl_$f
done
cd $R
LP_FUSED_NL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'])"
