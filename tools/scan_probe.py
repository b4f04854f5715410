#!/usr/bin/env python3
"""Latency of the literal-free scan kernel on request-sized texts (10k lines): the realistic
request vs uniform synthetic lines, to tell data-dependent cost (exact re-walks, long lines)
from fixed cost (LDS staging, launch). Medians of HIP-event timings."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from log_parser_amd.engine import Engine  # noqa: E402
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.ops import kernels as K  # noqa: E402
from log_parser_amd.native import N  # noqa: E402
from log_parser_amd.utils.config import Config, ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_log, realistic_library  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(1000, seed=7)
    eng = Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
    sp = eng.tabs["scan_passes"][0]
    texts = {
        "request": make_log(10_000, trig, seed=13, hit_rate=0.01),
        "x100": ("x" * 100 + "\n") * 10_000,
        "x300": ("x" * 300 + "\n") * 10_000,
        "lines10": ("abcdefghi\n") * 10_000,
        "one_line": "x" * 100 + "\n",
    }
    texts["bulk_1m25"] = texts["request"] * 125          # bulk path: 1024-thread blocks, 4-line runs
    out = {}
    for name, t in texts.items():
        data = t.encode()
        text, n = eng.stage_text(data)
        ls, ll = K.split_lines(text, n)
        L = ls.numel()
        buf = torch.empty(1 << 20, dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        lat = []
        for i in range(30 if L > 100_000 else 60):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            N.scan_multi(text.data_ptr(), n, ls.data_ptr(), ll.data_ptr(), L, sp, buf.data_ptr(), 1 << 20, cnt.data_ptr(),
                         eng.scan_grid(sp), st, True)
            b.record()
            torch.cuda.synchronize()
            if i >= 10:
                lat.append(a.elapsed_time(b) * 1e3)
        out[name] = {"lines": L, "us": round(float(np.median(lat)), 1), "hits_total": int(cnt.item())}
    out["lds_bytes"] = sp[1] * 4
    print(json.dumps(out))


if __name__ == "__main__":
    main()
