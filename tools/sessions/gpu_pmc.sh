#!/bin/bash
# rocprofv3 hardware-counter passes (kernel-trace/stats only: no sys/runtime/hip tracing with --pmc)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
export ENGINE_CONTEXT_ENGINE=mfma
ARGS="--steps 1 --warmup 1 --lines-per-gpu 2500000"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
           "VALUBusy VALUUtilization OccupancyPercent"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
  echo "PMC pass $i ok"
done
cd $R
timeout -k 10 500 python benchmarks/bench_configs.py concurrent > gpurun_out/cfg_concurrent.json 2> gpurun_out/cfg_concurrent.err && echo CONC_OK &&
timeout -k 10 600 python benchmarks/bench_configs.py stream --lines 100000000 --patterns 4000 > gpurun_out/cfg_stream.json 2> gpurun_out/cfg_stream.err && echo STREAM_OK
