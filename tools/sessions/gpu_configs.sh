#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
(cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1); echo "counters rc=$?"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --profile > gpurun_out/bench_profile.json 2> gpurun_out/bench_profile.err && echo PROFILE_OK &&
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > gpurun_out/cfg_single.json 2> gpurun_out/cfg_single.err && echo SINGLE_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK &&
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 100000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK
