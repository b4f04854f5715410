#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 100000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK
