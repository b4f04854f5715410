#!/bin/bash
# Round-2 evidence session: smoke, pytest -m gpu, headline bench, /parse breakdown, engine phases,
# request kernel trace, bulk kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r2m}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -20 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || exit 1
timeout -k 10 200 python tools/parse_breakdown.py --n 200 > $OUT/breakdown.json 2> $OUT/breakdown.err && echo BD_OK || exit 1
timeout -k 10 200 python tools/engine_phases.py --n 200 > $OUT/phases.json 2> $OUT/phases.err && echo PH_OK || exit 1
timeout -k 10 200 python tools/scan_probe.py > $OUT/scan_probe.json 2> $OUT/scan_probe.err && echo SP_OK || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/req -o req -- python3 $R/tools/request_trace.py --requests 200 > $R/$OUT/request_trace.json 2> $R/$OUT/request_trace.err && echo RT_OK || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 8 --warmup 2 --parse-requests 0 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err && echo PROF_OK || exit 1
cd $R
python tools/request_trace.py --db $OUT/req/req_results.db --requests 200 > $OUT/request_kernels.txt 2>&1 || true
