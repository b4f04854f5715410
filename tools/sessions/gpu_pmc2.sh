#!/bin/bash
# rocprofv3 hardware-counter passes over the headline bench (default DFA context engine), one
# counter group per run (no sys/runtime tracing together with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --lines-per-gpu 2500000 --parse-requests 0"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "VALUBusy VALUUtilization OccupancyPercent"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
  echo "PMC pass $i ok"
done
