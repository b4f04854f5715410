#!/bin/bash
# Round 3: BPG tests first, then the whole GPU suite, default bench, NFA engine A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_a}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bpg.py tests/test_backtrack.py > $OUT/pytest_bpg.log 2>&1 && echo BPG_OK || { tail -40 $OUT/pytest_bpg.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python tools/scan_ab.py --regexes 64 --lines 1000000 --engine all --reps 5 > $OUT/scan_ab.json 2>&1 && echo AB_OK || { tail -20 $OUT/scan_ab.json; exit 1; }
cat $OUT/scan_ab.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
