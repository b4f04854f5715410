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
# bench step kernel table (ingest serialised), request timeline, launch lag of one request
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 6 --warmup 2 --parse-requests 0 --no-overlap
db=$(find gpurun_out/prof_bench -name "*.db" | head -1)
run kstats 120 python3 tools/kstats_db.py "$db" 6 45 --median --marker k_nl_count --last 6 --timeline
find gpurun_out/prof_bench -name "*stats*" -exec cp {} gpurun_out/ \;
rm -rf gpurun_out/prof_bench
run lagprof 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/lag -o run -- \
  python3 tools/request_trace.py --requests 200 --java-shape-rate 0.01
run lag 120 python3 tools/launch_lag.py gpurun_out/lag --requests 200
rm -rf gpurun_out/lag
