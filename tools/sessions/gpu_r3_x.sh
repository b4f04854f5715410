#!/bin/bash
# Round 3: fewer small launches (granule memsets, no cat / fill kernels) + side-stream priority A/B
# (does k_pf_verify overlap k_scan_multi when the scan stream has high priority?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_x}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dp.py tests/test_post_bulk.py tests/test_gpu.py tests/test_bench.py > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for prio in 0 -1; do
  LP_SIDE_PRIORITY=$prio timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tl_$prio -o run -- python3 $R/bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > $R/$OUT/tl_$prio.log 2>&1 && echo TL_${prio}_OK || { tail -20 $R/$OUT/tl_$prio.log; exit 1; }
  DB=$(ls $R/$OUT/tl_$prio/*/run_results.db $R/$OUT/tl_$prio/run_results.db 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $DB --skip 3 > $R/$OUT/timeline_prio$prio.txt 2>&1 || true
  head -14 $R/$OUT/timeline_prio$prio.txt
  rm -rf $R/$OUT/tl_$prio
done
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'])"
