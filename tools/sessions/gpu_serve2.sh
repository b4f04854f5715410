#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 300 > gpurun_out/cfg_rest_gpu_native.json 2> gpurun_out/cfg_rest_gpu_native.err && echo NATIVE_OK &&
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 300 --http uvicorn > gpurun_out/cfg_rest_gpu_uvicorn.json 2> gpurun_out/cfg_rest_gpu_uvicorn.err && echo UVICORN_OK &&
timeout -k 10 300 python benchmarks/bench_configs.py rest --requests 100 > gpurun_out/cfg_rest_cpu_native.json 2> gpurun_out/cfg_rest_cpu_native.err && echo RESTCPU_OK
