#!/bin/bash
# Round 3: kernel traces of the current tree -- one 10k-line request (engine only) and the bulk step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o run -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/req.log 2>&1 && echo REQ_OK || { tail -20 $R/$OUT/req.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/bulk -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/bulk.log 2>&1 && echo BULK_OK || { tail -20 $R/$OUT/bulk.log; exit 1; }
cd $R
python tools/request_trace.py --db $(ls $OUT/req/*/run_results.db $OUT/req/run_results.db 2>/dev/null | head -1) --requests 200 > $OUT/req_kernels.txt 2>&1 || true
python tools/kstats_db.py $(ls $OUT/bulk/*/run_results.db $OUT/bulk/run_results.db 2>/dev/null | head -1) 7 45 --median > $OUT/bulk_kernels.txt 2>&1 || true
head -30 $OUT/req_kernels.txt; tail -3 $OUT/req.log
rm -rf $OUT/req $OUT/bulk
