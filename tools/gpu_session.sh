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
run rt 300 python -u tools/request_trace.py --requests 400 --java-shape-rate 0.01
run single 300 python -u benchmarks/bench_configs.py single
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run lagprof 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/lag -o run -- \
  python3 tools/request_trace.py --requests 200 --java-shape-rate 0.01
run lag 120 python3 tools/launch_lag.py gpurun_out/lag --requests 200
rm -rf gpurun_out/lag
run cprof 300 rocprofv3 --kernel-trace -d gpurun_out/cp -o run -- python3 benchmarks/bench_configs.py single --steps 8
run ctl 120 python3 tools/kstats_db.py $(find gpurun_out/cp -name "*.db" | head -1) 5 40 --marker k_nl_count --last 5 --timeline
rm -rf gpurun_out/cp
