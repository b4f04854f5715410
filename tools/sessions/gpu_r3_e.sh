#!/bin/bash
# Round 3: why does a world-1 RCCL group stall the ingest overlap? A/B of the suspects + traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-gpurun_out/r3_e}
mkdir -p $OUT
run() {  # name backend env...
  local name=$1; local be=$2; shift; shift
  timeout -k 10 200 env "$@" python bench.py --steps 12 --warmup 3 --parse-requests 0 --backend $be > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "FAIL $name"; tail -5 $OUT/b_$name.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name',d['backend'],d['ms_per_step'],d['device_ms_per_step_rank0'])"
}
run none none LP_X=0 && \
run nccl nccl LP_X=0 && \
run nccl_skipcoll nccl LP_DP_SKIP_WORLD1=1 && \
run nccl_lazy nccl LP_BENCH_LAZY_NCCL=1 && \
run nccl_nomon nccl TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 && \
run gloo1 gloo LP_X=0 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/prof_none -o run -- python3 $R/bench.py --steps 5 --warmup 2 --parse-requests 0 --backend none > $R/$OUT/prof_none.log 2>&1 && echo PROF_OK
