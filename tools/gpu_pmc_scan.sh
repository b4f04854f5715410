# PMC of the bench step's scan walk and prefilter (serialised step): LDS vs VALU vs waiting.
# Output: gpurun_out/pmc_scan/p{1,2}/... + gpurun_out/pmc_scan_summary.txt
# Run: gpurun -- bash tools/gpu_pmc_scan.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
for p in 1 2; do
  eval pmc=\$P$p
  timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "k_prefilter|k_scan_multi" \
    -d gpurun_out/pmc_scan/p$p -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --parse-requests 0 --no-overlap > gpurun_out/pmc_scan_p$p.log 2>&1
  rc=$?; echo "p$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_scan > gpurun_out/pmc_scan_summary.txt 2>&1
echo "summary rc=$?"
