#!/bin/bash
# round 2, first GPU pass: GPU tests, nccl world-1 bench (synthetic + realistic library "before")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --library synthetic --steps 10 --warmup 3 > $O/bench_synth.json 2> $O/bench_synth.err || { echo "bench synth failed"; tail -30 $O/bench_synth.err; exit 1; }
cat $O/bench_synth.json
timeout -k 10 300 python bench.py --library realistic --lines-per-gpu 2500000 --steps 3 --warmup 1 --parse-requests 10 > $O/bench_real_2m5.json 2> $O/bench_real.err || { echo "bench real failed"; tail -30 $O/bench_real.err; exit 1; }
cat $O/bench_real_2m5.json
