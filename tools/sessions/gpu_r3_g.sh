#!/bin/bash
# Round 3: confirm RCCL at world 1 as the bench default with >= 8 HIP hardware queues
# (utils/launch.ensure_hw_queues), smoke first; the driver-style bench (with /parse) last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_g}
mkdir -p $OUT
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "FAIL $name"; tail -5 $OUT/b_$name.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name',d['backend'],d.get('hip_hw_queues'),d['ms_per_step'],d['device_ms_per_step_rank0'],d.get('p50_parse_ms'),d.get('p99_parse_ms'))"
}
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
run auto --steps 12 --warmup 3 --parse-requests 0 && \
run none --steps 12 --warmup 3 --parse-requests 0 --backend none && \
run auto2 --steps 12 --warmup 3 --parse-requests 0 && \
run driver --steps 20 --warmup 5 || exit 1
