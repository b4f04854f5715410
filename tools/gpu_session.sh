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

cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run bprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bp -o run -- python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap
run btl 120 python3 tools/kstats_db.py $(find gpurun_out/bp -name "*.db" | head -1) 6 40 --marker k_nl_count --last 6 --timeline
rm -rf gpurun_out/bp
