#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent_e1.json 2> gpurun_out/cfg_concurrent_e1.err && echo CONC1_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent --engines 2 > gpurun_out/cfg_concurrent_e2.json 2> gpurun_out/cfg_concurrent_e2.err && echo CONC2_OK
