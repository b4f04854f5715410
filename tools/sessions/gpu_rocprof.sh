#!/bin/bash
# rocprofv3 kernel stats of the headline bench (3 timed steps) -> gpurun_out/prof/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --parse-requests ${PARSE_REQ:-0} > $R/gpurun_out/rocprof.log 2>&1 && echo ROCPROF_OK
