#!/bin/bash
# Host-side request overhead: cProfile of 200 engine requests, engine phases, /parse breakdown,
# headline bench (device-count + publish default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2p}
mkdir -p $OUT
timeout -k 10 200 python tools/cprof_request.py > $OUT/cprof.txt 2> $OUT/cprof.err && echo CPROF_OK || exit 1
timeout -k 10 200 python tools/engine_phases.py --n 300 > $OUT/phases.json 2> $OUT/phases.err && echo PH_OK || exit 1
timeout -k 10 200 python tools/parse_breakdown.py --n 300 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
