# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}

python - > gpurun_out/s_topo.log 2>&1 <<'PY'
import os
from log_parser_amd.utils.numa import l3_groups, gpu_numa_cpus, cpu_limits
a = os.sched_getaffinity(0)
print("allowed", len(a), "limits", cpu_limits(), "gpu0 node cpus", len(gpu_numa_cpus(0)))
print("l3 groups of gpu0 node cpus", [len(g) for g in l3_groups(gpu_numa_cpus(0) & a)][:16])
PY
for k in 1 2 3; do
  run l3_$k 300 python -u tools/parse_stages.py --n 400
  run nol3_$k 300 python -u tools/parse_stages.py --n 400 -D server.l3-affinity=false
done
run bench4 300 python -u bench.py --steps 10 --warmup 3
