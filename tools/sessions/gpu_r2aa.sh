#!/bin/bash
# CPU-backend speedups (AVX-512 host prefilter, K-way host context walk): GPU tests, REST CPU / GPU
# configs, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2aa}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python benchmarks/bench_configs.py rest --requests 200 > $OUT/cfg_rest_cpu.json 2> $OUT/cfg_rest_cpu.err && echo REST_CPU_OK || exit 1
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 300 > $OUT/cfg_rest_gpu.json 2> $OUT/cfg_rest_gpu.err && echo REST_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
