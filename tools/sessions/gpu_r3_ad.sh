#!/bin/bash
# Round 3: k_feat_cov with batched coverage loads and a uint16 LDS list -- tests first, whole GPU
# suite, step timeline (ingest not overlapped), bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_ad}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_post_bulk.py > $OUT/pytest_first.log 2>&1 && echo FIRST_OK || { tail -40 $OUT/pytest_first.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in noov; do
  X=""; [ $v = noov ] && X="--no-overlap"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$v -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 $X > $R/$OUT/tl_$v.log 2>&1 && echo TL_${v}_OK || { tail -20 $R/$OUT/tl_$v.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$v/*/run_results.db $R/$OUT/tl_$v/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 --marker k_nl_count > $R/$OUT/timeline_$v.txt 2>&1 || true
  python3 $R/tools/kstats_db.py $DB 5 60 --median --marker k_nl_count --last 5 > $R/$OUT/bulk_kernels_$v.txt 2>&1 || true
  head -1 $R/$OUT/timeline_$v.txt
  head -14 $R/$OUT/bulk_kernels_$v.txt
  rm -rf $R/$OUT/tl_$v
done
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'])"
