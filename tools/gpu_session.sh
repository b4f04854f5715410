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

run full_pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run full_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run full_bench 400 python -u bench.py
run single 300 python -u benchmarks/bench_configs.py single
run c5 300 python -u benchmarks/bench_configs.py concurrent_http --client-threads 8
run ps 300 python -u tools/parse_stages.py --n 400
run small 300 python -u tools/small_phases.py --requests 300
