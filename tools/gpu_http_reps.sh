# Config 5 over HTTP, repeated: 1 and 2 serving processes alternately, 3 times each (run-to-run
# variance on a shared host is large). Logs: gpurun_out/gh_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the box's CPU runs the AVX-512 block decoders this container lacks
timeout -k 10 300 python -u -m pytest tests/test_json_in.py -q -x > gpurun_out/gh_json_in.log 2>&1
rc=$?; echo "json_in rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for p in 1 2; do
    for ct in 8 4; do
      timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes $p --client-threads $ct \
        > gpurun_out/gh_p${p}_c${ct}_$i.log 2>&1
      rc=$?; echo "p$p c$ct rep$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
