#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 200 > gpurun_out/cfg_rest_gpu.json 2> gpurun_out/cfg_rest_gpu.err && echo RESTGPU_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK
