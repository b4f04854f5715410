#!/bin/bash
# Round 3: per-shape BPG vs MFMA NFA A/B (scan + candidate verify) and PMC passes of both engines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_o}
mkdir -p $OUT
timeout -k 10 400 python tools/nfa_ab.py --lines 1000000 --cands 20000 --reps 5 > $OUT/nfa_ab.jsonl 2> $OUT/nfa_ab.err && echo AB_OK || { tail -20 $OUT/nfa_ab.err; exit 1; }
cat $OUT/nfa_ab.jsonl
cd /tmp && export TMPDIR=/tmp
i=0
for eng in mfma bpg; do
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/$OUT/pmc_$eng/p$i -o run -- python3 $R/tools/nfa_ab.py --lines 250000 --cands 5000 --reps 1 --engine $eng --shapes bounded_gap,repeated_group > $R/$OUT/pmc_${eng}_$i.log 2>&1 || { echo "PMC $eng pass $i failed"; tail -5 $R/$OUT/pmc_${eng}_$i.log; exit 1; }
  done
done
cd $R
for eng in mfma bpg; do python3 tools/pmc_summary.py $OUT/pmc_$eng > $OUT/pmc_$eng.md 2>&1 || true; done
cat $OUT/pmc_mfma.md $OUT/pmc_bpg.md | cut -c1-400
rm -rf $OUT/pmc_mfma $OUT/pmc_bpg
