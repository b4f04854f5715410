# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}

bash tools/gpu_check.sh httpreps pmcscan || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
run pmc1n 180 rocprofv3 --pmc $P1 --kernel-include-regex "k_scan_multi|k_scan_rare" -d gpurun_out/pmc_scan_nodefer/p1 \
  -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parse-requests 0 --no-overlap --scan-defer-rare 0
run pmc2n 180 rocprofv3 --pmc $P2 --kernel-include-regex "k_scan_multi|k_scan_rare" -d gpurun_out/pmc_scan_nodefer/p2 \
  -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parse-requests 0 --no-overlap --scan-defer-rare 0
run pmcsumn 120 python3 tools/pmc_summary.py gpurun_out/pmc_scan_nodefer
