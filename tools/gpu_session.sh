# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}

mkdir -p gpurun_out/rehearsal
# world-8 rehearsal on the one GPU: 8 real rank processes, 12.5M lines each, gloo (host-staged)
run reh8 600 python -u bench.py --gpus 8 --ranks-per-gpu 8 --steps 3 --warmup 1 --parse-requests 0 \
  --phase-log gpurun_out/rehearsal/phases
# the same 8 shards concatenated, one rank (digest must equal)
run reh1 600 python -u bench.py --gpus 1 --lines-per-gpu 100000000 --steps 3 --warmup 1 --parse-requests 0
bash tools/gpu_check.sh pmcscan || exit 1
