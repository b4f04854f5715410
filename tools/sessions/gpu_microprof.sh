#!/bin/bash
# rocprofv3 kernel stats of tools/micro_latency.py (per-kernel durations of the request path)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/microprof -o run -- python3 $R/tools/micro_latency.py > $R/gpurun_out/microprof.log 2>&1 && echo MICROPROF_OK
