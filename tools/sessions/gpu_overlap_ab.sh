#!/bin/bash
# overlap A/B: per-step time vs process group / D2H stream (synthetic + realistic library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ovl
mkdir -p $O
for v in "--library synthetic" "--library synthetic --backend nccl" "--library synthetic --d2h-stream compute" "--library realistic"; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --parse-requests 0 $v > $O/b.json 2> $O/b.err || { echo "failed: $v"; tail -20 $O/b.err; exit 1; }
  echo "$v: $(grep -c . $O/b.json) stdout line(s): $(grep "^{" $O/b.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'],d['device_ms_per_step_rank0'],d['backend'],d['value'])")"
done
