#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/latprof -o run -- python3 $R/tools/latency_kernels.py 100 > $R/gpurun_out/latprof.log 2>&1 && echo LATPROF_OK
