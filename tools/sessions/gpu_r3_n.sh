#!/bin/bash
# Round 3: newline bitmask between the line-index passes -- GPU tests, kernel table of the last 5 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_stream.py tests/test_dp.py tests/test_pipeline.py > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
cd $R
python tools/kstats_db.py $(ls $OUT/bulk/*/run_results.db $OUT/bulk/run_results.db 2>/dev/null | head -1) 5 60 --median --marker k_nl_count --last 5 > $OUT/bulk_kernels.txt 2>&1 || true
cat $OUT/bulk_kernels.txt
rm -rf $OUT/bulk
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --parse-requests 0 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['matcher_counts_rank0'])"
