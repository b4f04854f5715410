#!/bin/bash
# Round 3: BPG kernels + shared-window serving on the GPU; A/B; bench; kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_b}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bpg.py tests/test_backtrack.py tests/test_multi_engine.py tests/test_resilience.py > $OUT/pytest_new.log 2>&1 && echo NEW_OK || { tail -60 $OUT/pytest_new.log; exit 1; }
timeout -k 10 300 python tools/scan_ab.py --regexes 64 --lines 1000000 --engine all --reps 5 > $OUT/scan_ab.json 2>&1 && echo AB_OK || { tail -20 $OUT/scan_ab.json; exit 1; }
tail -1 $OUT/scan_ab.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 > $R/$OUT/prof.log 2>&1 && echo PROF_OK || { tail -20 $R/$OUT/prof.log; exit 1; }
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
