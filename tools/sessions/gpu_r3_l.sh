#!/bin/bash
# Round 3: fingerprinted literal verify (k_pf_verify) -- GPU tests, request trace, bulk kernel table, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py tests/test_prefilter_tables.py tests/test_post.py tests/test_pipeline.py tests/test_bpg.py > $OUT/pytest_core.log 2>&1 && echo CORE_TESTS_OK || { tail -40 $OUT/pytest_core.log; exit 1; }
tail -1 $OUT/pytest_core.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/req -o run -- python3 $R/tools/request_trace.py --requests 300 > $R/$OUT/req.log 2>&1 && echo REQ_OK || { tail -20 $R/$OUT/req.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
cd $R
python tools/request_trace.py --db $(ls $OUT/req/*/run_results.db $OUT/req/run_results.db 2>/dev/null | head -1) --requests 300 > $OUT/req_kernels.txt 2>&1 || true
head -8 $OUT/req_kernels.txt; grep p50 $OUT/req.log | tail -1
python tools/kstats_db.py $(ls $OUT/bulk/*/run_results.db $OUT/bulk/run_results.db 2>/dev/null | head -1) 7 45 --median > $OUT/bulk_kernels.txt 2>&1 || true
head -12 $OUT/bulk_kernels.txt; tail -1 $OUT/bulk_kernels.txt
rm -rf $OUT/req $OUT/bulk
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'],d['matcher_counts_rank0'])"
