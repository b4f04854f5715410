# PMC A/B of the bench step's first kernels with the next step's H2D copy overlapping (the
# production schedule) and without it (--no-overlap): k_prefilter / k_nl_lines counters.
# Output: gpurun_out/pmc_ov/{on,off}/p{1,2}/...  Run: gpurun -- bash tools/gpu_pmc_overlap.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum"
for mode in on off; do
  extra=""; [ $mode = off ] && extra="--no-overlap"
  for p in 1 2; do
    eval pmc=\$P$p
    timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "k_prefilter|k_nl_lines|k_scan_multi" \
      -d gpurun_out/pmc_ov/$mode/p$p -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --parse-requests 0 $extra > gpurun_out/pmc_ov_${mode}_p$p.log 2>&1
    rc=$?; echo "$mode p$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
