#!/bin/bash
# Round 3: /parse tail A/B -- standalone server trace, bench with/without the world-1 RCCL group,
# server with HIP's default 4 hardware queues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_m}
mkdir -p $OUT
timeout -k 10 300 python tools/parse_tail.py --n 400 > $OUT/tail_standalone.txt 2>&1 && echo TAIL_OK || { tail -20 $OUT/tail_standalone.txt; exit 1; }
head -5 $OUT/tail_standalone.txt
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --parse-requests 400 "$@" > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "FAIL $name"; tail -5 $OUT/b_$name.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name',d['backend'],d['p50_parse_ms'],d['p99_parse_ms'],d['p50_engine_ms'],d['p99_engine_ms'])"
}
run nccl && run none --backend none && run nccl_srvq4 --server-env LP_HW_QUEUES=0 --server-env GPU_MAX_HW_QUEUES=4 && run nccl2 || exit 1
