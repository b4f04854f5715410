# Copy / kernel timeline of the 1B-line stream (config 4, 8 GiB chunks) -> gpurun_out/prof_stream/
# Run: gpurun -- bash tools/gpu_prof_stream.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_stream -o run -- \
  python3 benchmarks/bench_configs.py stream --chunk-mb 8192 > gpurun_out/prof_stream.log 2>&1
echo "prof rc=$?"
