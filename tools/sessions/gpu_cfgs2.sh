#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK &&
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > gpurun_out/cfg_single.json 2> gpurun_out/cfg_single.err && echo SINGLE_OK &&
timeout -k 10 300 python benchmarks/bench_configs.py rest --requests 100 > gpurun_out/cfg_rest.json 2> gpurun_out/cfg_rest.err && echo REST_OK &&
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 100000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK &&
timeout -k 10 900 python benchmarks/bench_configs.py stream --lines 1000000000 --patterns 4000 > gpurun_out/cfg_stream_1b.json 2> gpurun_out/cfg_stream_1b.err && echo STREAM1B_OK
