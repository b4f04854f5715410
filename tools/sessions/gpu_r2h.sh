#!/bin/bash
# scan A/B + kernel trace of the realistic bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd)
O=$R/gpurun_out/${OUT:-r2h}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 16 64; do
  timeout -k 10 120 python3 $R/tools/scan_ab.py --regexes $n --lines ${AB_LINES:-2500000} --engine dfa >> $O/ab.jsonl 2> $O/ab_$n.err || { echo "ab $n failed"; tail -20 $O/ab_$n.err; exit 1; }
done
cat $O/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --parse-requests 0 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
grep "^{" $O/prof.log | cut -c1-300
