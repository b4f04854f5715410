"""Kernel-level view of single-request latency: run N 10k-line /parse requests (1k patterns) so
that `rocprofv3 --kernel-trace --stats` attributes GPU time per kernel per request."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from log_parser_amd.engine import Engine  # noqa: E402
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.utils.config import Config, ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_library, make_log  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
sets, trig = make_library(1000, seed=7)
lib = CompiledLibrary(sets, ScoringParams())
req = make_log(10_000, trig, seed=13, hit_rate=0.01)
eng = Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
for _ in range(10):
    eng.analyze_batch_json([req])
lat = []
for _ in range(n):
    t = time.perf_counter()
    eng.analyze_batch_json([req])
    lat.append(time.perf_counter() - t)
print({"requests": n, "p50_ms": round(float(np.median(lat)) * 1e3, 3)})
