#!/bin/bash
# Quick GPU check: GPU tests, single-request latency breakdown, headline bench (short).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 240 python tools/latency_profile.py > gpurun_out/latency.log 2>&1 && echo LAT_OK &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --profile > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK
