# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}

run pytest 600 python -u -m pytest tests/test_java_shapes.py tests/test_backtrack.py tests/test_stream.py tests/test_regex.py \
  -m gpu -x -v --timeout 300 --timeout-method thread
run bench_la0 300 python -u bench.py --steps 10 --warmup 3 --parse-requests 0
run bench_la5 300 python -u bench.py --steps 10 --warmup 3 --parse-requests 0 --lookaround-patterns 5
run bench_bt3 300 python -u bench.py --steps 10 --warmup 3 --parse-requests 0 --bt-patterns 3
run nfa_lib 300 python -u tools/nfa_ab.py --library realistic --lines 1000000
run nfa_shapes 400 python -u tools/nfa_ab.py --lines 1000000
bash tools/gpu_check.sh pmcscan || exit 1
