# Round-end rehearsal: the whole GPU test suite, smoke(), the bench and its kernel table.
# Run: gpurun -- bash tools/gpu_full.sh   (logs: gpurun_out/full_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/full_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/full_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/full_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/full_bench.log | cut -c1-400
