# GPU-box validation session. Logs under gpurun_out/. Steps (default: all, in this order):
#   tests   the regex / serving / MFMA GPU tests
#   scantest  the literal-free scan kernel's GPU tests (bulk + request variants, CRLF) and the kernel tests
#   scan    scan-group A/B (32 vs 64 members per multi-regex DFA)
#   nfa     MFMA vs BPG A/B per regex shape (tools/nfa_ab.py)
#   bench   bench.py (headline, 1 GPU)
#   http    config 5 over HTTP: 1 and 2 serving processes (stage timelines), and the front end alone
#   stream  config 4: 1B-line stream, auto (HBM-sized) chunks and 256 MiB chunks (same digest)
#   configs config 2 (1M lines, 256 patterns, realistic library) and config 1 (CPU-only /parse)
# Run: gpurun -- bash tools/gpu_check.sh [step ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
steps="${*:-tests scan nfa bench http}"

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/gc_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

for s in $steps; do
  case $s in
    tests)
      run tests 900 python -u -m pytest tests/test_bpg.py tests/test_java_shapes.py tests/test_backtrack.py \
        tests/test_nfa.py tests/test_regex.py tests/test_serve_procs.py tests/test_stream.py -m gpu -x -v --durations=15 --timeout 300 \
        --timeout-method thread ;;
    scantest)
      run scantest 600 python -u -m pytest tests/test_scan_multi.py tests/test_gpu.py -m gpu -x -q --timeout 300 \
        --timeout-method thread ;;
    scan)
      run scan32 300 python -u tools/scan_ab.py --regexes 46 --engine dfa --group-regs 32 --lines 12500000
      run scan64 300 python -u tools/scan_ab.py --regexes 46 --engine dfa --group-regs 64 --lines 12500000 ;;
    nfa)
      run nfa_ab 400 python -u tools/nfa_ab.py --lines 1000000 ;;
    bench)
      run bench 600 python -u bench.py --steps 10 --warmup 3 ;;
    http)
      run http1 300 python -u benchmarks/bench_configs.py concurrent_http --timeline \
        --server-log gpurun_out/gc_http1_srv.log
      run http2 300 python -u benchmarks/bench_configs.py concurrent_http --processes 2 --timeline \
        --server-log gpurun_out/gc_http2_srv.log
      run ceiling 300 python -u tools/http_ceiling.py --requests 10000 --io 2,8 ;;
    stream)
      run stream_auto 600 python -u benchmarks/bench_configs.py stream
      run stream_8g 600 python -u benchmarks/bench_configs.py stream --chunk-mb 8192
      run stream_256 600 python -u benchmarks/bench_configs.py stream --chunk-mb 256 ;;
    reqtrace)
      # one 10k-line request: wall p50 and the kernel timeline, library with / without the Java shapes
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      for j in 0 0.01; do
        run rt_wall_$j 300 python -u tools/request_trace.py --requests 400 --java-shape-rate $j
        run rt_prof_$j 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/rt_prof_$j -o run -- \
          python3 tools/request_trace.py --requests 200 --java-shape-rate $j
        db=$(find gpurun_out/rt_prof_$j -name "*.db" | head -1)
        run rt_sum_$j 120 python3 tools/request_trace.py --db "$db" --requests 200
      done ;;
    configs)
      run single 600 python -u benchmarks/bench_configs.py single
      run rest 600 python -u benchmarks/bench_configs.py rest ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
