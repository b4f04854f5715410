#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 100000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK &&
timeout -k 10 900 python benchmarks/bench_configs.py stream --lines 1000000000 --patterns 4000 > gpurun_out/cfg_stream_1b.json 2> gpurun_out/cfg_stream_1b.err && echo STREAM1B_OK
