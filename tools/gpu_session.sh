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

run pytest 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v -k "run_document or sharded_single or fetch_publish" \
  --timeout 200 --timeout-method thread
run single 300 python -u benchmarks/bench_configs.py single
run phases 300 python -u tools/engine_phases.py --n 200
bash tools/gpu_check.sh reqtrace prof || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run prof_nodefer 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nodefer -o run -- \
  python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap --scan-defer-rare 0
db=$(find gpurun_out/prof_nodefer -name "*.db" | head -1)
run kstats_nodefer 120 python3 tools/kstats_db.py "$db" 6 45 --median --marker k_nl_count --last 6
bash tools/gpu_check.sh httpreps || exit 1
