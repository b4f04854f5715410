#!/bin/bash
# Request-path iteration: GPU tests of the touched kernels, request kernel trace, /parse breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2l}
TESTS=${TESTS:-tests/test_gpu.py tests/test_scan_multi.py}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/pytest.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 200 python tools/engine_phases.py > $OUT/phases.json 2> $OUT/phases.err && cat $OUT/phases.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err || exit 1
cd $R
python tools/request_trace.py --db $(ls $OUT/req/*/req_results.db 2>/dev/null | head -1 || echo $OUT/req/req_results.db) --requests 200 > $OUT/request_kernels.txt 2>&1; head -20 $OUT/request_kernels.txt
