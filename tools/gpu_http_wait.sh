# Config 5: does holding batches open (engine.batch.max-wait-ms) help 2 serving processes, which
# otherwise pass the shared window back and forth in small batches (profiles/r4_d)?
# Run: gpurun -- bash tools/gpu_http_wait.sh   (logs: gpurun_out/hw_*.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  for cfg in "2 0" "2 2" "2 5" "1 0" "1 2"; do
    set -- $cfg
    timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes $1 --client-threads 8 \
      --server-opt=-Dengine.batch.max-wait-ms=$2 > gpurun_out/hw_p$1_w$2_$rep.log 2>&1
    rc=$?; echo "p$1 wait$2 rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
