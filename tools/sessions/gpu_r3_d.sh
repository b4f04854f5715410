#!/bin/bash
# Round 3 configs: config 5 over HTTP (10k connections), resident 50 GiB re-analysis, config 4
# with HBM-sized chunks (equality vs 256 MiB chunks on 100M lines, then 1B lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/r3_d}
mkdir -p $OUT
B="python benchmarks/bench_configs.py"
timeout -k 10 400 $B concurrent_http --requests 10000 > $OUT/cfg_concurrent_http.json 2> $OUT/cfg_concurrent_http.err && echo HTTP_OK || { tail -20 $OUT/cfg_concurrent_http.err; exit 1; }
cat $OUT/cfg_concurrent_http.json
timeout -k 10 400 $B concurrent_http --requests 10000 --engines 2 > $OUT/cfg_concurrent_http_e2.json 2> $OUT/cfg_concurrent_http_e2.err && echo HTTP2_OK || { tail -20 $OUT/cfg_concurrent_http_e2.err; exit 1; }
cat $OUT/cfg_concurrent_http_e2.json
timeout -k 10 300 $B stream --lines 100000000 --patterns 4000 --chunk-mb 256 > $OUT/cfg_stream_100M_256M.json 2> $OUT/s1.err && echo S1_OK || { tail -20 $OUT/s1.err; exit 1; }
timeout -k 10 300 $B stream --lines 100000000 --patterns 4000 --chunk-mb 4096 > $OUT/cfg_stream_100M_4G.json 2> $OUT/s2.err && echo S2_OK || { tail -20 $OUT/s2.err; exit 1; }
python - <<PY
import json
a=json.load(open("$OUT/cfg_stream_100M_256M.json")); b=json.load(open("$OUT/cfg_stream_100M_4G.json"))
print("256M", a["seconds"], a["chunks"], a["topk_digest"], "| 4G", b["seconds"], b["chunks"], b["topk_digest"])
print("EQUAL" if (a["summary"]==b["summary"] and a["topk_digest"]==b["topk_digest"] and a["events"]==b["events"]) else "DIFFERENT")
PY
timeout -k 10 400 $B stream --lines 1000000000 --patterns 4000 > $OUT/cfg_stream_1B.json 2> $OUT/s3.err && echo S3_OK || { tail -20 $OUT/s3.err; exit 1; }
cat $OUT/cfg_stream_1B.json
timeout -k 10 500 $B resident --gb 50 > $OUT/cfg_resident_50G.json 2> $OUT/r.err && echo RES_OK || { tail -20 $OUT/r.err; exit 1; }
cat $OUT/cfg_resident_50G.json
