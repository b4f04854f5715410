#!/bin/bash
# /parse tail breakdown (server-side receive / validate / queue / engine of the slowest requests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2v}
mkdir -p $OUT
timeout -k 10 300 python tools/parse_tail.py --n 400 > $OUT/parse_tail.json 2> $OUT/parse_tail.err && echo TAIL_OK || { tail -20 $OUT/parse_tail.err; exit 1; }
