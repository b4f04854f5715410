#!/bin/bash
# eviction inside k_fetch A/B (engine p50 / p99, alternating runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2ee}
mkdir -p $OUT
T="timeout -k 10 200 python tools/request_trace.py --requests 600"
LP_RUNNER_EVICT_IN_FETCH=1 $T > $OUT/ab.jsonl 2>/dev/null && echo A1 || exit 1
LP_RUNNER_EVICT_IN_FETCH=0 $T >> $OUT/ab.jsonl 2>/dev/null && echo B1 || exit 1
LP_RUNNER_EVICT_IN_FETCH=1 $T >> $OUT/ab.jsonl 2>/dev/null && echo A2 || exit 1
LP_RUNNER_EVICT_IN_FETCH=0 $T >> $OUT/ab.jsonl 2>/dev/null && echo B2 || exit 1
