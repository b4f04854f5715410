#!/usr/bin/env python3
"""Host-side phase timing of one 10k-line request through Engine.analyze_batch_json (the
p50_engine_ms path): wall time spent in each Python-level phase, medians over N requests. Phases
that end in a host read (match_and_hits' counter read, the results D2H) include the GPU time
still in flight at that point."""
import argparse
import json
import os
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--lines", type=int, default=10_000)
    ap.add_argument("-D", action="append", default=[], help="config override key=value (A/B runs)")
    ap.add_argument("--bytes", action="store_true", help="request body as bytes (default: str, as bench.py)")
    args = ap.parse_args()
    import torch
    from log_parser_amd import engine as E
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_log, realistic_library
    from log_parser_amd.utils.numa import bind_to_gpu_numa
    bind_to_gpu_numa(0)                     # as bench.py: pinned stages on the GPU's socket
    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(1000, seed=7)
    eng = E.Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides=dict([("engine.device", "cuda:0")] + [tuple(d.split("=", 1)) for d in args.D])), device=dev)
    logs = make_log(args.lines, trig, seed=13, hit_rate=0.01)
    if args.bytes:
        logs = logs.encode()
    acc = defaultdict(list)
    cur = {}

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                cur[label] = cur.get(label, 0.0) + time.perf_counter() - t
        setattr(obj, name, g)

    wrap(eng, "pack_batch", "pack")
    wrap(eng, "_stage_docs", "pack.stage_docs")
    wrap(eng, "device_batch", "device_batch")
    wrap(eng, "_run_native", "device.run_native")
    wrap(eng, "_host_keys", "device.host_keys")
    wrap(eng, "_stage_h2d", "stage_h2d")
    wrap(eng.upload.__class__, "__call__", "upload")
    wrap(K, "match_and_hits", "match_and_hits(+read)")
    wrap(K, "post_events", "post_events")
    wrap(K, "results_buffer", "results_buffer")
    wrap(eng, "finish", "finish")
    wrap(eng, "commit_frequency", "commit_freq")
    wrap(eng, "_results_to_host", "results_d2h")
    wrap(eng, "emit_batch", "emit")
    wrap(eng, "release_batch", "release")
    wrap(eng, "freq_carry", "freq_carry")
    for i in range(args.n + 10):
        cur.clear()
        t = time.perf_counter()
        eng.analyze_batch_json([logs])
        tot = time.perf_counter() - t
        if i >= 10:
            for k, v in cur.items():
                acc[k].append(v)
            acc["total"].append(tot)
    out = {k: round(float(np.median(v)) * 1e3, 4) for k, v in acc.items()}
    out["overrides"] = args.D
    print(json.dumps(out))


if __name__ == "__main__":
    main()
