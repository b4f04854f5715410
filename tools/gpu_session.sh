# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_bpg.py tests/test_java_shapes.py tests/test_serve_procs.py tests/test_backtrack.py tests/test_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/s_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/request_trace.py --requests 400 --java-shape-rate 0.01 > gpurun_out/s_rt.log 2>&1 || exit 1
tail -1 gpurun_out/s_rt.log | cut -c1-100
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/s_bench.log 2>&1
echo "bench rc=$?"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bt-patterns 4 --parse-requests 0 > gpurun_out/s_bench_bt.log 2>&1
echo "bench bt rc=$?"
