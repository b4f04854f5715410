# Copy-engine probe, queued copies (tools/copy_engine_probe.py --backlog) under a kernel +
# memory-copy trace -> gpurun_out/copy_backlog_summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/copy_backlog -o run -- \
  python3 tools/copy_engine_probe.py --backlog > gpurun_out/copy_backlog.log 2>&1
echo "probe rc=$?"
db=$(find gpurun_out/copy_backlog -name "*.db" | head -1)
timeout -k 10 120 python3 tools/copy_trace_summary.py "$db" > gpurun_out/copy_backlog_summary.txt 2>&1
echo "summary rc=$?"
