#!/usr/bin/env python3
"""Per-request stage means of sequential 10k-line POST /parse requests inside the server process
(GET /admin/stages before / after): the native front end's receive / validate / queue / handoff /
send and the pump thread's pack / device / emit / dispatch / complete, next to the client's wall
p50 -- where the server-side engine time (pump pick-up -> response queued) goes, compared with the
same request through Engine.analyze_batch_json in-process (tools/engine_phases.py).

    python tools/parse_stages.py --n 300
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("-D", action="append", default=[], help="server config override key=value")
    a = ap.parse_args()
    import numpy as np
    from log_parser_amd.utils import restbench
    from log_parser_amd.utils.synth import make_log, realistic_library
    sets, trig = realistic_library(1000, seed=7)
    server = restbench.ServerProcess(restbench.write_library(sets), a.device, http="native",
                                     extra=[f"-D{d}" for d in a.D])
    try:
        if not server.wait_ready():
            raise SystemExit("server did not come up")
        logs = make_log(10_000, trig, seed=13, hit_rate=0.01)
        server.parse_latencies(logs, 30, warmup=5)
        b = restbench.collect_stages(server.port)
        t0 = time.perf_counter()
        lat = np.array(server.parse_latencies(logs, a.n, warmup=0)) * 1e3
        wall = time.perf_counter() - t0
        e = restbench.collect_stages(server.port)
    finally:
        server.stop()
    (pid, before), = b.items()
    after = e[pid]
    n = after["requests"] - before["requests"]
    per = {}
    for grp in ("pump", "pipeline"):
        for k, v in after.get(grp, {}).items():
            per[f"{grp}.{k}_us"] = round(1e6 * (v - before.get(grp, {}).get(k, 0.0)) / max(n, 1), 1)
    nat = {}
    an, bn = after["native"], before["native"]
    for k, v in an.items():
        if k.endswith("_s"):
            cnt = {"receive_s": "parse", "validate_s": "parse", "queue_s": "drained", "handoff_s": "responses",
                   "send_s": "sent"}.get(k, "parse")
            nat[k[:-2] + "_us"] = round(1e6 * (v - bn.get(k, 0.0)) / max(an.get(cnt, 0) - bn.get(cnt, 0), 1), 1)
    nat["prefetched"] = an.get("prefetched", 0) - bn.get("prefetched", 0)
    print(json.dumps({"requests": n, "p50_ms": round(float(np.median(lat)), 3),
                      "p99_ms": round(float(np.percentile(lat, 99)), 3), "wall_s": round(wall, 3),
                      "native": nat, "server_threads": per, "overrides": a.D}), flush=True)


if __name__ == "__main__":
    main()
