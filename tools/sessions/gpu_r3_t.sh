#!/bin/bash
# Round 3 (re-entry baseline): whole GPU suite, bench, and PMC passes of the bulk step's big kernels
# (prefilter with the Teddy tier, union-DFA scan, literal verify).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 && echo TESTS_OK || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'],d['matcher_counts_rank0'])"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "k_prefilter|k_scan_multi|k_pf_verify" --output-format csv -d $R/$OUT/pmc/p$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --parse-requests 0 --backend none > $R/$OUT/pmc_$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/$OUT/pmc_$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_bulk.md 2>&1 || true
cut -c1-600 $OUT/pmc_bulk.md
rm -rf $OUT/pmc
