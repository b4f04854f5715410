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

run gt 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run small 300 python -u tools/small_phases.py --requests 300
run rt 300 python -u tools/request_trace.py --requests 400 --java-shape-rate 0.01
run eph 300 python -u tools/engine_phases.py --n 300
run rt2 300 python -u tools/request_trace.py --requests 400 --java-shape-rate 0.01
run ps 300 python -u tools/parse_stages.py --n 400
