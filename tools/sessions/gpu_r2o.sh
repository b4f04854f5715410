#!/bin/bash
# Request-path A/B session: GPU tests, engine p50 for host-count / device-count + publish /
# device-count without publish / blit copies (HSA_ENABLE_SDMA=0) / cached-store packer, and a
# kernel trace of the device-count + publish runner.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
T="timeout -k 10 200 python tools/request_trace.py --requests 400"
$T > $OUT/ab.jsonl 2>/dev/null && echo hc_ok || exit 1
$T --device-counts >> $OUT/ab.jsonl 2>/dev/null && echo dc_ok || exit 1
LP_RUNNER_PUBLISH=0 $T --device-counts >> $OUT/ab.jsonl 2>/dev/null && echo dc_nopub_ok || exit 1
HSA_ENABLE_SDMA=0 $T --device-counts >> $OUT/ab.jsonl 2>/dev/null && echo dc_nosdma_ok || exit 1
LP_PACK_NT=0 $T --device-counts >> $OUT/ab.jsonl 2>/dev/null && echo dc_packcached_ok || exit 1
$T --device-counts >> $OUT/ab.jsonl 2>/dev/null && echo dc_again_ok || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/reqdc -o req -- python3 $R/tools/request_trace.py --requests 200 --device-counts > $R/$OUT/request_trace_dc.json 2> $R/$OUT/request_trace_dc.err && echo RTDC_OK || exit 1
HSA_ENABLE_SDMA=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/reqns -o req -- python3 $R/tools/request_trace.py --requests 200 --device-counts > $R/$OUT/request_trace_ns.json 2> $R/$OUT/request_trace_ns.err && echo RTNS_OK || exit 1
cd $R
python tools/request_trace.py --db $OUT/reqdc/req_results.db --requests 200 > $OUT/request_kernels_dc.txt 2>&1 || true
python tools/request_trace.py --db $OUT/reqns/req_results.db --requests 200 > $OUT/request_kernels_nosdma.txt 2>&1 || true
rm -rf $OUT/reqdc $OUT/reqns
