#!/bin/bash
# Round-2 refresh of the other BASELINE configs on the current tree (each step time-limited).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/cfg_r2}
mkdir -p $OUT
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > $OUT/cfg_single.json 2> $OUT/cfg_single.err && echo SINGLE_OK && cat $OUT/cfg_single.json || exit 1
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu --requests 200 > $OUT/cfg_rest_gpu.json 2> $OUT/cfg_rest_gpu.err && echo REST_OK && cat $OUT/cfg_rest_gpu.json || exit 1
timeout -k 10 300 python benchmarks/bench_configs.py rest --requests 100 > $OUT/cfg_rest_cpu.json 2> $OUT/cfg_rest_cpu.err && echo REST_CPU_OK && cat $OUT/cfg_rest_cpu.json || exit 1
timeout -k 10 500 python benchmarks/bench_configs.py concurrent --requests 10000 > $OUT/cfg_concurrent.json 2> $OUT/cfg_concurrent.err && echo CONC_OK && cat $OUT/cfg_concurrent.json || exit 1
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 1000000000 --patterns 4000 > $OUT/cfg_stream.json 2> $OUT/cfg_stream.err && echo STREAM_OK && cat $OUT/cfg_stream.json || exit 1
