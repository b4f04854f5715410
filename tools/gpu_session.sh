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

run pytest 600 python -u -m pytest tests/test_bpg.py tests/test_java_shapes.py tests/test_backtrack.py tests/test_gpu.py \
  tests/test_scan_multi.py \
  -m gpu -x -v --timeout 200 --timeout-method thread
bash tools/gpu_check.sh reqtrace || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run rts_prof 300 rocprofv3 --kernel-trace -d gpurun_out/rts_prof -o run -- \
  python3 tools/request_trace.py --requests 200 --java-shape-rate 0.01 --split-verify
db=$(find gpurun_out/rts_prof -name "*.db" | head -1)
run rts_sum 120 python3 tools/request_trace.py --db "$db" --requests 200
run phases 300 python -u tools/engine_phases.py --n 200
run single 300 python -u benchmarks/bench_configs.py single
bash tools/gpu_check.sh singletrace || exit 1
run bench 400 python -u bench.py --steps 10 --warmup 3
run bench_bt 400 python -u bench.py --steps 10 --warmup 3 --bt-patterns 4 --parse-requests 0
bash tools/gpu_check.sh pmcscan || exit 1
