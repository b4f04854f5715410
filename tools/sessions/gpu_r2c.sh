#!/bin/bash
# scan engine A/B (multi-DFA scan groups vs MFMA NFA) + PMC counters of both kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd)
O=$R/gpurun_out/r2c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 16 32 64 128; do
  timeout -k 10 120 python3 $R/tools/scan_ab.py --regexes $n --lines 2500000 >> $O/ab.jsonl 2> $O/ab_$n.err || { echo "ab $n failed"; tail -20 $O/ab_$n.err; exit 1; }
done
cat $O/ab.jsonl
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "VALUBusy VALUUtilization OccupancyPercent"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 $R/tools/scan_ab.py --regexes 64 --lines 1000000 --reps 2 > $O/pmc$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  echo "PMC pass $i ok"
done
