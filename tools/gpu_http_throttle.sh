# Config 5, repeated, with the cgroup's CFS throttling recorded per burst: is the run-to-run spread
# (profiles/r4_d) quota throttling? Logs: gpurun_out/ht_*.log, cgroup files: gpurun_out/ht_cgroup.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
{ cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpuset.cpus.effective 2>&1; nproc; } > gpurun_out/ht_cgroup.txt || true
for rep in 1 2 3 4; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py concurrent_http --processes 1 --client-threads 8 \
    > gpurun_out/ht_p1_$rep.log 2>&1
  rc=$?; echo "p1 rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
