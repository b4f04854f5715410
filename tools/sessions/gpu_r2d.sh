#!/bin/bash
# scan_multi v2 (line runs): GPU tests, A/B vs MFMA, PMC, realistic bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd)
O=$R/gpurun_out/${OUT:-r2d}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for n in 16 64 128; do
  timeout -k 10 120 python3 $R/tools/scan_ab.py --regexes $n --lines 2500000 --engine ${ENG:-both} >> $O/ab.jsonl 2> $O/ab_$n.err || { echo "ab $n failed"; tail -20 $O/ab_$n.err; exit 1; }
done
cat $O/ab.jsonl
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "VALUBusy VALUUtilization OccupancyPercent"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 $R/tools/scan_ab.py --regexes 64 --lines 1000000 --reps 2 --engine dfa > $O/pmc$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
timeout -k 10 300 python $R/bench.py --library realistic --steps 10 --warmup 3 > $O/bench_real.json 2> $O/bench_real.err || { echo "bench real failed"; tail -30 $O/bench_real.err; exit 1; }
cat $O/bench_real.json
