# Config 5: front-end IO threads (server.io-threads) x 4 runs each. Logs: gpurun_out/hio_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4; do
  for io in 4 6 8; do
    timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes 1 --client-threads 8 \
      --server-opt=-Dserver.io-threads=$io > gpurun_out/hio_${io}_$rep.log 2>&1
    rc=$?; echo "io$io rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
