#!/usr/bin/env python3
"""Where the time of one POST /parse (10k-line, ~1 MB body) goes, measured piece by piece:

  loopback  : raw TCP round trip of the same byte count to a Python echo thread (kernel floor)
  http_400  : native front end in this process, body with "pod": null (full receive + JSON
              validation + 400 response, no engine)
  decode    : N.parse_pod_request on the body (validation + unescape, in process)
  engine    : Engine.analyze_batch_json([bytes]) in process (pack, H2D, kernels, D2H, JSON emit)
  parse_raw : the full request through a server process, raw-socket client (pre-built request)
  parse_lib : the same through http.client (what bench.py used in round 1 / early round 2)

Prints one JSON line of medians (ms)."""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(fn, n, warm=10):
    for _ in range(warm):
        fn()
    lat = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        lat.append(time.perf_counter() - t)
    return round(float(np.median(lat)) * 1e3, 3)


def loopback_ms(nbytes, n):
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen()

    def srv():
        c, _ = ls.accept()
        buf = bytearray(nbytes)
        mv = memoryview(buf)
        while True:
            got = 0
            while got < nbytes:
                k = c.recv_into(mv[got:], nbytes - got)
                if k == 0:
                    return
                got += k
            c.sendall(b"ok")
    threading.Thread(target=srv, daemon=True).start()
    s = socket.create_connection(ls.getsockname())
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    msg = b"x" * nbytes

    def rt():
        s.sendall(msg)
        s.recv(2)
    r = med(rt, n)
    s.close()
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--lines", type=int, default=10_000)
    args = ap.parse_args()
    from log_parser_amd.utils import restbench
    from log_parser_amd.utils.synth import make_log, realistic_library
    sets, trig = realistic_library(1000, seed=7)
    server = restbench.ServerProcess(restbench.write_library(sets), args.device, http="native")
    logs = make_log(args.lines, trig, seed=13, hit_rate=0.01)
    body = json.dumps({"pod": {"metadata": {"name": "bench"}}, "logs": logs}).encode()
    out = {"body_bytes": len(body)}
    try:
        if not server.wait_ready():          # compiled and idle before anything is timed
            raise SystemExit("server did not come up")
        out["loopback"] = loopback_ms(len(body), args.n)
        from log_parser_amd.native import N
        hs = N.HttpServer("127.0.0.1", 0, 1, 1 << 30, 60.0)
        cl = restbench.RawClient("127.0.0.1", hs.port)
        bad = json.dumps({"logs": logs, "pod": None}).encode()
        out["http_400"] = med(lambda: cl.post(bad), args.n)
        cl.close()
        hs.stop()
        out["decode"] = med(lambda: N.parse_pod_request(body), args.n)
        import torch
        from log_parser_amd.engine import Engine
        from log_parser_amd.models.compiled import CompiledLibrary
        from log_parser_amd.utils.config import Config, ScoringParams
        dev = torch.device(args.device)
        eng = Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides={"engine.device": str(dev)}),
                     device=dev)
        lb = logs.encode()
        out["engine"] = med(lambda: eng.analyze_batch_json([lb]), args.n)
        raw = np.array(server.parse_latencies(logs, args.n)) * 1e3
        out["parse_raw"] = round(float(np.median(raw)), 3)
        out["parse_raw_p90_p99_max"] = [round(float(np.percentile(raw, q)), 3) for q in (90, 99, 100)]
        worst = np.argsort(raw)[-6:][::-1]
        out["parse_raw_worst"] = [[int(i), round(float(raw[i]), 3)] for i in worst]     # (index, ms)
        out["parse_lib"] = round(float(np.median(server.parse_latencies(logs, args.n, client="http.client"))) * 1e3, 3)
        out["response_bytes"] = len(server.post(body)[1])
    finally:
        server.stop()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
