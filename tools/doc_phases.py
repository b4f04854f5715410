"""Host-side phases of config 2's resident document step (Engine.run_document): wall-clock marks at
the entry / exit of the orchestration calls between the line index's count read and the matcher
launches, medians over R runs. Shows where the Python set-up keeps the GPU waiting (the kernel
timeline puts ~100 us between the line-count read and the first scan launch).

    python tools/doc_phases.py --lines 1000000 --runs 30
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=1_000_000)
    ap.add_argument("--patterns", type=int, default=256)
    ap.add_argument("--runs", type=int, default=30)
    a = ap.parse_args()
    import torch
    from log_parser_amd import engine as E
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.native import N
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_log, realistic_library

    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(a.patterns, seed=5)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = E.Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
    data = make_log(a.lines, trig, seed=9, hit_rate=0.004).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    text = t.to(dev)
    marks = []

    def wrap(owner, name, label):
        f = getattr(owner, name)

        def g(*args, **kw):
            marks.append((label + ">", time.perf_counter()))
            r = f(*args, **kw)
            marks.append((label + "<", time.perf_counter()))
            return r
        setattr(owner, name, g)

    wrap(K, "split_lines", "split_lines")
    wrap(K, "EarlyPrefilter", "early_pf")
    wrap(K, "_line_index_dev", "line_index")
    wrap(E.Segments, "scalar", "segments")
    wrap(E.Engine, "prepare", "prepare")
    wrap(E.Engine, "_ev_tables", "ev_tables")
    wrap(E.Engine, "host_hits", "host_hits")
    wrap(K, "match_and_hits", "match_and_hits")
    wrap(K, "line_block_index", "blk_index")
    wrap(N, "scan_multi", "scan_launch")
    wrap(K, "post_events", "post_events")
    wrap(E.Engine, "finish", "finish")
    wrap(N, "line_index_dev", "n_line_index")
    wrap(N, "prefilter_dev", "n_prefilter")
    wrap(K, "_pf_events", "pf_events")
    wrap(E.Engine, "freq_carry", "freq_carry")
    for _ in range(5):
        eng.run_document(text, len(data))
    torch.cuda.synchronize()
    per = {}
    for _ in range(a.runs):
        marks.clear()
        t0 = time.perf_counter()
        eng.run_document(text, len(data))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        seen = set()
        for lab, ts in marks:
            if lab in seen:
                continue
            seen.add(lab)
            per.setdefault(lab, []).append((ts - t0) * 1e6)
        per.setdefault("return", []).append((t1 - t0) * 1e6)
    out = {k: round(statistics.median(v), 1) for k, v in sorted(per.items(), key=lambda kv: statistics.median(kv[1]))}
    print(json.dumps({"lines": a.lines, "us_from_start_median": out}), flush=True)


if __name__ == "__main__":
    main()
