#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
rm -rf gpurun_out/pmc_mfma && mkdir -p gpurun_out/pmc_mfma
cd /tmp && export TMPDIR=/tmp
export ENGINE_CONTEXT_ENGINE=mfma
ARGS="--steps 1 --warmup 1 --lines-per-gpu 2500000 --parse-requests 0"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc_mfma/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_mfma/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc_mfma/p$i.log; exit 1; }
  echo "PMC pass $i ok"
done
