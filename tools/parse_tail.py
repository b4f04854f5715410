"""Where the slow POST /parse requests spend their time: a server process with server.trace-requests
on (receive / validate per request from the C++ front end, queue / engine per request from the pump), N
sequential 10k-line requests from the raw client; prints the median and the slowest requests with
their server-side breakdown (requests are sequential, so trace line i is request i).

    python tools/parse_tail.py --n 400
"""
import argparse
import json
import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    import numpy as np
    from log_parser_amd.utils import restbench
    from log_parser_amd.utils.synth import make_log, realistic_library
    sets, trig = realistic_library(1000, seed=7)
    log_path = os.path.join(tempfile.mkdtemp(prefix="lp-tail-"), "server.log")
    server = restbench.ServerProcess(restbench.write_library(sets), a.device, http="native", log_path=log_path,
                                     extra=["-Dserver.trace-requests=true"])
    try:
        if not server.wait_ready():
            raise SystemExit("server did not come up")
        logs = make_log(10_000, trig, seed=13, hit_rate=0.01)
        lat = np.array(server.parse_latencies(logs, a.n, warmup=20)) * 1e3
    finally:
        server.stop()
    text = open(log_path).read()
    http = [tuple(float(x) for x in m) for m in
            re.findall(r"lp-http-trace bytes \d+ receive_us ([\d.]+) recvs (\d+) wakeups (\d+) validate_us ([\d.]+)", text)]
    pump = [tuple(float(x) for x in m) for m in re.findall(r"lp-parse-trace queue_us ([\d.-]+) engine_us ([\d.]+)", text)]
    # the last n records belong to the timed requests (warm-up requests come first)
    http, pump = http[-a.n:], pump[-a.n:]
    rows = []
    for i in np.argsort(lat)[::-1][:10]:
        r = {"i": int(i), "ms": round(float(lat[i]), 3)}
        if len(http) == a.n:
            r.update(receive_us=http[i][0], recvs=int(http[i][1]), wakeups=int(http[i][2]), validate_us=http[i][3])
        if len(pump) == a.n:
            r.update(queue_us=pump[i][0], engine_us=pump[i][1])
        rows.append(r)
    med = {"ms": round(float(np.median(lat)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3)}
    if len(http) == a.n:
        med.update(receive_us=float(np.median([h[0] for h in http])), validate_us=float(np.median([h[3] for h in http])))
    if len(pump) == a.n:
        med.update(queue_us=float(np.median([p[0] for p in pump])), engine_us=float(np.median([p[1] for p in pump])))
    print(json.dumps({"median": med, "slowest": rows, "records": [len(http), len(pump)]}, indent=1), flush=True)


if __name__ == "__main__":
    main()
