#!/bin/bash
# Round 3: RCCL world-1 stall -- hardware-queue hypothesis: copy stream created before vs after the
# process group; more HW queues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_f}
mkdir -p $OUT
run() {  # name backend env...
  local name=$1; local be=$2; shift; shift
  timeout -k 10 200 env "$@" python bench.py --steps 12 --warmup 3 --parse-requests 0 --backend $be > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "FAIL $name"; tail -5 $OUT/b_$name.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name',d['backend'],d['ms_per_step'],d['device_ms_per_step_rank0'],d['matcher_counts_rank0'])"
}
run none none LP_X=0 && \
run nccl_early nccl LP_X=0 && \
run nccl_late nccl LP_BENCH_LATE_COPY_STREAM=1 && \
run nccl_late_q8 nccl LP_BENCH_LATE_COPY_STREAM=1 GPU_MAX_HW_QUEUES=8 && \
run nccl_early2 nccl LP_X=0 || exit 1
