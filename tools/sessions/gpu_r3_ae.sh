#!/bin/bash
# Round 3: PMC of the bulk step's mid-size kernels (context features, BPG verify, line index, summary).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_ae}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "k_feat_cov|k_bpg_dedupe_all|k_nl_count|k_nl_lines|k_summ_level|k_dedupe_verify" --output-format csv -d $R/$OUT/pmc/p$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --parse-requests 0 --backend none > $R/$OUT/pmc_$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/$OUT/pmc_$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_mid.md 2>&1 || true
cut -c1-700 $OUT/pmc_mid.md
rm -rf $OUT/pmc
