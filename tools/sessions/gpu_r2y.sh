#!/bin/bash
# Rank sort in the single-workgroup stages + 64-line feature blocks + k_fetch only for request-sized
# uploads: GPU tests, request trace, concurrent burst (fetch on / off), feature-block A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2y}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
T="timeout -k 10 200 python tools/request_trace.py --requests 400"
$T > $OUT/ab.jsonl 2>/dev/null && echo rt_ok || exit 1
LP_FC_REQUEST_LINES=256 $T >> $OUT/ab.jsonl 2>/dev/null && echo rt256_ok || exit 1
timeout -k 10 500 python benchmarks/bench_configs.py concurrent --requests 10000 > $OUT/cfg_concurrent.json 2> $OUT/cfg_concurrent.err && echo CONC_OK || exit 1
LP_RUNNER_FETCH=0 timeout -k 10 500 python benchmarks/bench_configs.py concurrent --requests 10000 > $OUT/cfg_concurrent_nofetch.json 2> $OUT/cfg_concurrent_nofetch.err && echo CONC0_OK || exit 1
LP_RUNNER_PUBLISH=0 timeout -k 10 500 python benchmarks/bench_configs.py concurrent --requests 10000 > $OUT/cfg_concurrent_nopub.json 2> $OUT/cfg_concurrent_nopub.err && echo CONCP_OK || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RTP_OK || exit 1
cd $R
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
rm -rf $OUT/req
