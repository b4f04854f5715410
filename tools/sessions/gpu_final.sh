#!/bin/bash
# End-of-round evidence: PMC counter passes on the headline kernels (default engine) + the other
# BASELINE configs (single 1M-line request, REST on GPU, concurrent burst, 1B-line stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/pmc
ARGS="--steps 1 --warmup 1 --lines-per-gpu 2500000 --parse-requests 0"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "VALUBusy VALUUtilization OccupancyPercent"; do
  i=$((i+1))
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1) || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
  echo "PMC pass $i ok"
done
timeout -k 10 400 python benchmarks/bench_configs.py single --steps 5 > gpurun_out/cfg_single.json 2> gpurun_out/cfg_single.err && echo SINGLE_OK &&
timeout -k 10 300 python benchmarks/bench_configs.py rest_gpu > gpurun_out/cfg_rest_gpu.json 2> gpurun_out/cfg_rest_gpu.err && echo REST_OK &&
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK &&
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 1000000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK
