#!/usr/bin/env python3
"""Where the request path's single-workgroup kernels spend their time: phase clocks
(wall_clock64, 100 MHz on gfx950) written by k_hits_small / k_events_small, or the fused
k_request_tail (its score / record / publish phases too) (N.set_small_profile)
over R 10k-line requests, medians in microseconds.

    python tools/small_phases.py --requests 200
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HITS = ["compact", "sort", "dedupe+compact", "csr+events scan"]
EVENTS = ["init", "sort1", "post", "sort2", "ranks+coverage"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=200)
    ap.add_argument("--lines", type=int, default=10_000)
    ap.add_argument("--java-shape-rate", type=float, default=0.01)
    ap.add_argument("--mhz", type=float, default=100.0, help="wall_clock64 rate")
    a = ap.parse_args()
    import torch
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.native import N
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_log, realistic_library
    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(1000, seed=7, java_shape_rate=a.java_shape_rate)
    eng = Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
    logs = make_log(a.lines, trig, seed=13, hit_rate=0.01)
    for _ in range(10):
        eng.analyze_batch_json([logs])
    buf = torch.zeros(16, dtype=torch.int64, device=dev)
    N.set_small_profile(buf.data_ptr())
    ph = {k: [] for k in HITS + EVENTS + ["hits kernel", "events kernel"]}
    tail = {k: [] for k in ("tail: score", "tail: record", "tail: publish", "tail kernel")}
    live, nev = [], []
    try:
        for _ in range(a.requests):
            buf.zero_()
            eng.analyze_batch_json([logs])
            torch.cuda.synchronize()
            t = buf.cpu().tolist()
            us = 1.0 / a.mhz
            for i, k in enumerate(HITS):
                ph[k].append((t[i + 1] - t[i]) * us)
            for i, k in enumerate(EVENTS):
                ph[k].append((t[9 + i] - t[8 + i]) * us)
            ph["hits kernel"].append((t[4] - t[0]) * us)
            ph["events kernel"].append((t[13] - t[8]) * us)
            live.append(t[5])
            nev.append(t[14])
            if t[15]:       # the fused k_request_tail ran (score / record / publish stamps)
                tail["tail: score"].append((t[6] - t[13]) * us)
                tail["tail: record"].append((t[7] - t[6]) * us)
                tail["tail: publish"].append((t[15] - t[7]) * us)
                tail["tail kernel"].append((t[15] - t[0]) * us)
    finally:
        N.set_small_profile(0)
    out = {k: round(statistics.median(v), 2) for k, v in list(ph.items()) + list(tail.items()) if v}
    out["live_keys"] = statistics.median(live)
    out["events"] = statistics.median(nev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
