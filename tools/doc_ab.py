"""Same-box A/B of config 2's resident document step (Engine.run_document) for one host-side
ordering switch: the early literal prefilter launched before (``early_first``) or after the line
count's copy is set up. Alternates the two in rounds so box drift hits both.

    python tools/doc_ab.py --rounds 6 --steps 30
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from log_parser_amd import engine as E
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_log, realistic_library

    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(256, seed=7)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = E.Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
    data = make_log(a.lines, trig, seed=5, hit_rate=0.004, aux_rate=0.01, stack_rate=0.01).encode()
    text, n = eng.stage_text(data)

    def split(early_first):
        def f(text, nbytes):
            box = []
            ls, ll = K.split_lines(text, nbytes, before_read=lambda: box.append(eng.prefilter_early(text, nbytes)),
                                   early_first=early_first)
            return ls, ll, (box[0] if box else None)
        return f

    res = {"early_first": [], "after_copy": []}
    for _ in range(a.rounds):
        for label, ef in (("early_first", True), ("after_copy", False)):
            eng.split_with_prefilter = split(ef)
            for _ in range(3):
                eng.run_document(text, n)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.run_document(text, n)
            torch.cuda.synchronize()
            res[label].append((time.perf_counter() - t0) / a.steps * 1e3)
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 4), "runs_ms": [round(x, 4) for x in v]}
                      for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
