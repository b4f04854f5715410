# A/B of the fused line index (engine.fused-line-index: the prefilter's read of the text also
# writes the newline counts/masks, no k_nl_count) on the bench step, with kernel tables.
# Run: gpurun -- bash tools/gpu_ab_fused.sh   (logs: gpurun_out/ab_fused_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab_fused_off.log 2>&1 && echo "off rc=0" &&
ENGINE_FUSED_LINE_INDEX=true timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab_fused_on.log 2>&1 &&
echo "on rc=0" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in off on; do
  e=false; [ $v = on ] && e=true
  ENGINE_FUSED_LINE_INDEX=$e timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_prof_$v -o run -- \
    python3 bench.py --steps 6 --warmup 2 --parse-requests 0 > gpurun_out/ab_prof_$v.log 2>&1 || exit 1
  db=$(find gpurun_out/ab_prof_$v -name "*.db" | head -1)
  python3 tools/kstats_db.py "$db" 6 45 --median --marker k_prefilter --last 6 --timeline > gpurun_out/ab_fused_${v}_kernels.txt 2>&1
  echo "prof $v rc=$?"
done
