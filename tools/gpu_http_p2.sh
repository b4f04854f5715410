# Config 5 with 2 serving processes x 5 runs (after the stage pre-sizing). Logs: gpurun_out/hp2_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4 5; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes 2 --client-threads 8 \
    > gpurun_out/hp2_$rep.log 2>&1
  rc=$?; echo "p2 rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
