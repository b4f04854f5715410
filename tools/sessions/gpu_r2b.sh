#!/bin/bash
# round 2: scan groups + Teddy tier on the GPU: tests, benches (both libraries), kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --library realistic --steps 10 --warmup 3 > $O/bench_real.json 2> $O/bench_real.err || { echo "bench real failed"; tail -30 $O/bench_real.err; exit 1; }
cat $O/bench_real.json
timeout -k 10 300 python bench.py --library synthetic --steps 10 --warmup 3 --parse-requests 0 > $O/bench_synth.json 2> $O/bench_synth.err || { echo "bench synth failed"; tail -30 $O/bench_synth.err; exit 1; }
cat $O/bench_synth.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_real -o run -- python bench.py --library realistic --steps 3 --warmup 1 --parse-requests 0 > $O/prof_real.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof_real.log; exit 1; }
find $O/prof_real -name "*kernel_stats.csv" | head -3
