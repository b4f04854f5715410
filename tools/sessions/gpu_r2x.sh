#!/bin/bash
# /parse after quick-ack + pump spin + logging after respond: tail trace, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2x}
mkdir -p $OUT
timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/tail.json 2> $OUT/tail.err && echo TAIL_OK || exit 1
LP_HTTP_PUMP_SPIN_US=0 timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/tail_nospin.json 2> $OUT/tail_nospin.err && echo TAIL0_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --parse-requests 400 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
timeout -k 10 200 python tools/parse_breakdown.py --n 300 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
