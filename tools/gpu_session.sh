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

run pytest 800 python -u -m pytest tests/test_bpg.py tests/test_java_shapes.py tests/test_backtrack.py tests/test_gpu.py \
  tests/test_scan_multi.py tests/test_summarize.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread
run probe 300 python -u tools/bpg_probe.py --lens 32,128,512
bash tools/gpu_check.sh reqtrace || exit 1
run phases 300 python -u tools/engine_phases.py --n 200
run single 300 python -u benchmarks/bench_configs.py single
bash tools/gpu_check.sh singletrace || exit 1
run bench 400 python -u bench.py --steps 10 --warmup 3
run bench_bt 400 python -u bench.py --steps 10 --warmup 3 --bt-patterns 4 --parse-requests 0
bash tools/gpu_check.sh prof || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run pmcl 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_scan_multi" \
  -d gpurun_out/pmc_lds/p1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parse-requests 0 --no-overlap
