# Config 5 repeated with the server's stage timeline (which stage stretches in a slow run?)
# Logs: gpurun_out/htl_*.log (JSON line last; timeline on stderr lines "pid ...")
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4 5; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes 1 --client-threads 8 --timeline \
    > gpurun_out/htl_$rep.log 2>&1
  rc=$?; echo "rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
