#!/bin/bash
# /parse tail A/B: server TCP receive knobs (baseline / quick-ack / 4 MB SO_RCVBUF / pump spin).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r2w}
mkdir -p $OUT
sysctl net.core.rmem_max net.ipv4.tcp_rmem net.ipv4.tcp_wmem > $OUT/sysctl.txt 2>&1 || true
timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/base.json 2> $OUT/base.err && echo BASE_OK || exit 1
LP_HTTP_QUICKACK=1 timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/quickack.json 2> $OUT/quickack.err && echo QA_OK || exit 1
LP_HTTP_RCVBUF=4194304 timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/rcvbuf.json 2> $OUT/rcvbuf.err && echo RB_OK || exit 1
LP_HTTP_SPIN_US=2000 timeout -k 10 250 python tools/parse_tail.py --n 400 > $OUT/spin.json 2> $OUT/spin.err && echo SPIN_OK || exit 1
