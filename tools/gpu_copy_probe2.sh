# Is the bench's H2D a blit kernel only under a kernel-only trace? The probe under --kernel-trace
# alone, then the bench step under --kernel-trace + --memory-copy-trace.
# Run: gpurun -- bash tools/gpu_copy_probe2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/copy_probe_k -o run -- \
  python3 tools/copy_engine_probe.py > gpurun_out/copy_probe_k.log 2>&1 && echo "probe-k rc=0" &&
{ db=$(find gpurun_out/copy_probe_k -name "*.db" 2>/dev/null | head -1); [ -z "$db" ] && echo "probe-k: no kernels traced (no blit copies)" ||
  timeout -k 10 120 python3 tools/copy_trace_summary.py "$db" > gpurun_out/copy_probe_k_summary.txt 2>&1; true; } &&
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/copy_bench -o run -- \
  python3 bench.py --steps 6 --warmup 2 --parse-requests 0 > gpurun_out/copy_bench.log 2>&1 && echo "bench rc=0" &&
db=$(find gpurun_out/copy_bench -name "*.db" | head -1) &&
timeout -k 10 120 python3 tools/copy_trace_summary.py "$db" > gpurun_out/copy_bench_summary.txt 2>&1 &&
timeout -k 10 120 python3 tools/kstats_db.py "$db" 6 45 --median --marker k_prefilter --last 6 --timeline \
  > gpurun_out/copy_bench_kernels.txt 2>&1
echo "done rc=$?"
