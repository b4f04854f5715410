#!/bin/bash
# serving pipeline: GPU tests, 10k-concurrent burst (1 engine) with stage timeline, one-batch
# stage profile, REST latency (native front end)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent --timeline > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK &&
timeout -k 10 400 python tools/conc_profile.py > gpurun_out/conc_profile.log 2>&1 && echo CONCPROF_OK &&
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 300 > gpurun_out/cfg_rest_gpu_native.json 2> gpurun_out/cfg_rest_gpu_native.err && echo NATIVE_OK
