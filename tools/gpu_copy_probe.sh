# Copy-engine probe (tools/copy_engine_probe.py) under a kernel + memory-copy trace; the summary
# (which cases became blit kernels) -> gpurun_out/copy_probe_summary.txt
# Run: gpurun -- bash tools/gpu_copy_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/copy_probe -o run -- \
  python3 tools/copy_engine_probe.py > gpurun_out/copy_probe.log 2>&1
echo "probe rc=$?"
db=$(find gpurun_out/copy_probe -name "*.db" | head -1)
timeout -k 10 120 python3 tools/copy_trace_summary.py "$db" > gpurun_out/copy_probe_summary.txt 2>&1
echo "summary rc=$?"
