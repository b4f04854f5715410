#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2bb}
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo B1_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo B2_OK || exit 1
