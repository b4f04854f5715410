# A/B: lanes per gram hit of the bulk literal verify (k_pf_verify<L>), serialised bench step under a
# kernel trace -> gpurun_out/pv_<L>_kernels.txt (+ the bench line in pv_<L>.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in 4 2 1; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$L -o run -- \
    python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap --pf-verify-lanes $L > gpurun_out/pv_$L.log 2>&1
  rc=$?; echo "lanes $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
  db=$(find gpurun_out/pv_$L -name "*.db" | head -1)
  python3 tools/kstats_db.py "$db" 6 45 --median --marker k_nl_count --last 6 > gpurun_out/pv_${L}_kernels.txt 2>&1
done
