#!/bin/bash
# Round-2 end-of-session evidence: smoke, pytest -m gpu, headline bench, kernel table, request trace and
# the other BASELINE configs (single 1M-line request, REST GPU/CPU, 10k concurrent burst, 1B-line stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > $OUT/cfg_single.json 2> $OUT/cfg_single.err && echo SINGLE_OK || exit 1
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 200 > $OUT/cfg_rest_gpu.json 2> $OUT/cfg_rest_gpu.err && echo REST_OK || exit 1
timeout -k 10 300 python benchmarks/bench_configs.py rest --requests 100 > $OUT/cfg_rest_cpu.json 2> $OUT/cfg_rest_cpu.err && echo REST_CPU_OK || exit 1
timeout -k 10 500 python benchmarks/bench_configs.py concurrent --requests 10000 > $OUT/cfg_concurrent.json 2> $OUT/cfg_concurrent.err && echo CONC_OK || exit 1
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 1000000000 --patterns 4000 > $OUT/cfg_stream.json 2> $OUT/cfg_stream.err && echo STREAM_OK || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 8 --warmup 2 --parse-requests 0 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err && echo PROF_OK || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RT_OK || exit 1
cd $R
python tools/kstats_db.py $OUT/prof/run_results.db 10 30 --median > $OUT/kernel_table.txt 2>&1 || true
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
rm -rf $OUT/req $OUT/prof
