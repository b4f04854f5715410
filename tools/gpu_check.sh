# GPU-box validation session: regex / serving GPU tests, scan-group A/B, bench, config-5 HTTP (1 and 2
# serving processes) and the front-end ceiling. Logs under gpurun_out/. Run: gpurun -- bash tools/gpu_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_bpg.py tests/test_java_shapes.py tests/test_backtrack.py tests/test_nfa.py tests/test_regex.py tests/test_serve_procs.py -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread > gpurun_out/gpu2_regex.log 2>&1
rc=$?; echo "regex tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/scan_ab.py --regexes 46 --engine dfa --group-regs 16 > gpurun_out/gpu3_scan16.log 2>&1
rc=$?; echo "scan16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/scan_ab.py --regexes 46 --engine dfa --group-regs 32 > gpurun_out/gpu3_scan32.log 2>&1
rc=$?; echo "scan32 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/nfa_ab.py --lines 1000000 > gpurun_out/gpu2_nfa_ab.log 2>&1
rc=$?; echo "nfa_ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/gpu2_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --server-log gpurun_out/gpu2_http_srv1.log > gpurun_out/gpu2_http.log 2>&1
rc=$?; echo "http rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes 2 --server-log gpurun_out/gpu2_http_srv2.log > gpurun_out/gpu2_http2.log 2>&1
rc=$?; echo "http2 rc=$rc"
timeout -k 10 300 python -u tools/http_ceiling.py --requests 10000 --io 2,8 > gpurun_out/gpu2_ceiling.log 2>&1
rc=$?; echo "ceiling rc=$rc"
