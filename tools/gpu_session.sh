# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}

for k in 1 2 3; do
  run c5new_$k 300 python -u benchmarks/bench_configs.py concurrent_http --client-threads 8
  run c5always_$k 300 python -u benchmarks/bench_configs.py concurrent_http --client-threads 8 --server-opt=-Dserver.io-decode-max-conns=-1
  run c5r5_$k 300 python -u ab_old/benchmarks/bench_configs.py concurrent_http --client-threads 8
done
run ps 300 python -u tools/parse_stages.py --n 400
