# Ad-hoc GPU session of the current milestone (edited per call). Logs: gpurun_out/s_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {   # run NAME SECONDS CMD... : stop the session at the first failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/s_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/s_${name}.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}

for k in 1 2 3; do
  run dnew_$k 300 python -u tools/doc_ab.py --rounds 2 --steps 30
  run dold_$k 300 python -u ab_old/tools/doc_ab.py --rounds 2 --steps 30
done
