# GPU-box validation session. Logs under gpurun_out/. Steps (default: all, in this order):
#   tests   the regex / serving / MFMA GPU tests
#   scantest  the literal-free scan kernel's GPU tests (bulk + request variants, CRLF) and the kernel tests
#   scan    scan-group A/B (32 vs 64 members per multi-regex DFA)
#   nfa     MFMA vs BPG A/B per regex shape (tools/nfa_ab.py)
#   bench   bench.py (headline, 1 GPU)
#   http    config 5 over HTTP: 1 and 2 serving processes (stage timelines), and the front end alone
#   stream  config 4: 1B-line stream, auto (HBM-sized) chunks and 256 MiB chunks (same digest)
#   configs config 2 (1M lines, 256 patterns, realistic library) and config 1 (CPU-only /parse)
#   singletrace  config 2 kernel timeline (the whole-document step is the last one traced)
#   reqtrace  one 10k-line request: wall p50 + kernel timeline, library with / without Java shapes
#   splitverify  request path with the DFA / BPG candidate verification split, one BPG walk's cost
#   prof    kernel table of the bench step (rocprofv3 kernel trace, serialised ingest)
#   pmcbpg  PMC counters of one lean BPG walk (two passes)
#   pmcscan PMC counters of the scan walk and prefilter (two counter passes)
#   httpreps  config 5, 1 and 2 processes, 5 runs each: stage / connection timelines, thread states
#   full    round-end rehearsal: the whole GPU suite, smoke(), the bench
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
    splitverify)
      # request path with DFA and BPG candidates verified in two launches (each half's time), and
      # one BPG walk's cost per program (tools/bpg_probe.py)
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      for j in 0 0.01; do
        run sv_prof_$j 300 rocprofv3 --kernel-trace -d gpurun_out/sv_prof_$j -o run -- \
          python3 tools/request_trace.py --requests 200 --java-shape-rate $j --split-verify
        db=$(find gpurun_out/sv_prof_$j -name "*.db" | head -1)
        run sv_sum_$j 120 python3 tools/request_trace.py --db "$db" --requests 200
        rm -rf gpurun_out/sv_prof_$j
      done
      run bpg_probe 300 python3 tools/bpg_probe.py --lens 32,128,512 --java-shape-rate 0.01 ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- \
        python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap
      db=$(find gpurun_out/prof_bench -name "*.db" | head -1)
      run kstats 120 python3 tools/kstats_db.py "$db" 6 45 --median --marker k_nl_count --last 6 --timeline ;;
    pmcscan)
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      # four counters per pass (larger passes were refused on this pool in rounds 5 and 6)
      P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"
      P2="SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"
      P4="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
      k=1
      for P in "$P1" "$P2" "$P3" "$P4"; do
        run pmc$k 180 rocprofv3 --pmc $P --kernel-include-regex "k_prefilter|k_scan_multi|k_scan_rare" \
          -d gpurun_out/pmc_scan/p$k -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 \
          --parse-requests 0 --no-overlap --gen-workers 0
        k=$((k + 1))
      done
      run pmcsum 120 python3 tools/pmc_summary.py gpurun_out/pmc_scan ;;
    pmcbpg)
      # PMC of ONE lean BPG walk (tools/bpg_probe.py, 512-byte line): instructions and waits per walk
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      run pmcbpg1 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
        SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex "k_bpg_dedupe_all" -d gpurun_out/pmc_bpg/p1 -o run \
        --output-format csv -- python3 tools/bpg_probe.py --lens 512 --reps 3
      run pmcbpg2 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-include-regex "k_bpg_dedupe_all" \
        -d gpurun_out/pmc_bpg/p2 -o run --output-format csv -- python3 tools/bpg_probe.py --lens 512 --reps 3 ;;
    httpreps)
      # config 5, 1 and 2 serving processes, 5 runs each: stage + per-connection timelines and the
      # serving threads' states sampled every 1 ms (run-to-run spread, the slow mode's cause)
      for np in 1 2; do
        for rep in 1 2 3 4 5; do
          run htl_p${np}_$rep 300 python -u benchmarks/bench_configs.py concurrent_http --processes $np \
            --client-threads 8 --timeline --sample-threads
        done
      done ;;
    full)
      run full_pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
      run full_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
      run full_bench 300 python -u bench.py ;;
    singletrace)
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      run single_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_single -o run -- \
        python3 benchmarks/bench_configs.py single --steps 20
      db=$(find gpurun_out/prof_single -name "*.db" | head -1)
      run single_kstats 120 python3 tools/kstats_db.py "$db" 20 40 --median --marker k_nl_count --last 20 --timeline ;;
    configs)
      run single 600 python -u benchmarks/bench_configs.py single
      run rest 600 python -u benchmarks/bench_configs.py rest ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
