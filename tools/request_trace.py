"""Single-request path breakdown (the p50_engine_ms of bench.py): R requests of L lines through
``Engine.analyze_batch_json`` one at a time, wall time per request; run under
``rocprofv3 --kernel-trace --memory-copy-trace`` and summarise with ``--db`` to see how much of a
request is GPU kernels, copies, or host/launch gaps.

    python tools/request_trace.py --lines 10000 --requests 200
    python tools/request_trace.py --db gpurun_out/x/run_results.db --requests 200
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(args):
    import torch
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_log, realistic_library
    from log_parser_amd.utils.numa import bind_to_gpu_numa
    bind_to_gpu_numa(0)                     # as bench.py and the server: pinned stages on the GPU's socket
    dev = torch.device("cuda", 0)
    if args.split_verify:                   # k_cand_verify + the BPG walk as two launches (diagnostic)
        from log_parser_amd.native import N
        N.set_cand_verify_split(True)
    sets, trig = realistic_library(args.patterns, seed=7, java_shape_rate=args.java_shape_rate)
    lib = CompiledLibrary(sets, ScoringParams())
    ov = {"engine.device": "cuda:0"}
    if args.device_counts:
        ov["engine.runner-device-counts"] = True
    eng = Engine(lib, Config.load(overrides=ov), device=dev)
    logs = make_log(args.lines, trig, seed=13, hit_rate=0.01)
    for _ in range(20):
        eng.analyze_batch_json([logs])
    torch.cuda.synchronize()
    wall = []
    for _ in range(args.requests):
        t0 = time.perf_counter()
        eng.analyze_batch_json([logs])
        wall.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"lines": args.lines, "requests": args.requests, "java_shape_rate": args.java_shape_rate,
                      "library": lib.summary(), "p50_ms": round(statistics.median(wall), 3),
                      "p99_ms": round(sorted(wall)[int(0.99 * (len(wall) - 1))], 3)}), flush=True)


def summarise(args):
    import sqlite3
    db = sqlite3.connect(args.db)
    ks = db.execute("select name, start, end from kernels order by start").fetchall()
    try:
        cs = db.execute("select start, end from memory_copies order by start").fetchall()
    except sqlite3.Error:
        cs = []
    ev = sorted([(s, e, n) for n, s, e in ks] + [(s, e, "<copy>") for s, e in cs])
    # one k_prefilter launch per request: a request = from one to the next (steady state)
    marks = [x[0] for x in ev if "k_prefilter" in x[2]]
    groups = []
    for a, b in zip(marks, marks[1:]):
        groups.append([x for x in ev if a <= x[0] < b])
    groups = groups[-args.requests:]
    spans, busy, nk, nc = [], [], [], []
    per_name = {}
    for g in groups:
        spans.append((max(y[1] for y in g) - g[0][0]) / 1e3)     # first kernel .. last end
        busy.append(sum(y[1] - y[0] for y in g) / 1e3)
        nk.append(sum(1 for y in g if y[2] != "<copy>"))
        nc.append(sum(1 for y in g if y[2] == "<copy>"))
        for y in g:
            per_name.setdefault(y[2][:70], []).append((y[1] - y[0]) / 1e3)
    n = len(groups)
    print(json.dumps({"requests": n, "span_us_p50": round(statistics.median(spans), 1),
                      "busy_us_p50": round(statistics.median(busy), 1), "kernels_per_request": statistics.median(nk),
                      "copies_per_request": statistics.median(nc)}))
    for name, d in sorted(per_name.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"{sum(d) / n:8.1f} us/req  {len(d) / n:5.1f}/req  {name}")
    # timeline of the median-span request: start offset, duration and the idle gap before each op
    if groups:
        med = sorted(range(n), key=lambda i: spans[i])[n // 2]
        g = groups[med]
        t0, prev_end = g[0][0], g[0][0]
        print(f"timeline of request {med} (span {spans[med]:.1f} us): offset_us dur_us gap_us name")
        for s, e, name in g:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {max(0, s - prev_end) / 1e3:7.1f}  {name[:60]}")
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=10_000)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--requests", type=int, default=200)
    ap.add_argument("--db", default="")
    ap.add_argument("--java-shape-rate", type=float, default=0.01,
                    help="share of Java-shape primaries in the realistic library (0 = the round-3 library)")
    ap.add_argument("--split-verify", action="store_true",
                    help="verify DFA and BPG candidates in two launches (shows each half in a trace)")
    ap.add_argument("--device-counts", action="store_true", help="runner device-count mode (no mid-batch read)")
    a = ap.parse_args()
    summarise(a) if a.db else run(a)
