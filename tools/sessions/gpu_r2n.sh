#!/bin/bash
# Request-path session: GPU tests (runner single-copy upload), request traces in host-count and
# device-count mode, /parse breakdown, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RT_OK || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/reqdc -o req -- python3 $R/tools/request_trace.py --requests 200 --device-counts > $R/$OUT/request_trace_dc.json 2> $R/$OUT/request_trace_dc.err && echo RTDC_OK || exit 1
cd $R
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
python tools/request_trace.py --db $OUT/reqdc/req_results.db --requests 200 > $OUT/request_kernels_dc.txt 2>&1 || true
rm -rf $OUT/req $OUT/reqdc
timeout -k 10 200 python tools/request_trace.py --requests 300 > $OUT/rt_plain.json 2>&1 && echo RTP_OK || exit 1
timeout -k 10 200 python tools/request_trace.py --requests 300 --device-counts > $OUT/rt_plain_dc.json 2>&1 && echo RTPDC_OK || exit 1
timeout -k 10 200 python tools/parse_breakdown.py --n 200 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
