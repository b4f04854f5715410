# Kernel table of the bench step (rocprofv3 kernel trace, rocpd database) -> gpurun_out/prof_bench/
# --no-overlap: under the profiler the HIP runtime can turn the overlapped H2D into a blit kernel
# that shares the CUs with the step (profiles/r4_c); serialised, the kernel times are the step's own.
# Run: gpurun -- bash tools/gpu_prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find gpurun_out/prof_bench -name "*.db" | head -1)
python3 tools/kstats_db.py "$db" 6 45 --median --marker k_nl_count --last 6 > gpurun_out/prof_bench_kernels.txt 2>&1
echo "kstats rc=$?"
