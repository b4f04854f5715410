"""Single-request /parse latency breakdown (10k-line log, 1k patterns): p50 without tracing,
per-stage HIP-event timings (engine.trace), and a torch.profiler op table (launch/sync overhead)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from log_parser_amd.engine import Engine  # noqa: E402
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.utils.config import Config, ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_library, make_log  # noqa: E402


def main():
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    sets, trig = make_library(1000, seed=7)
    lib = CompiledLibrary(sets, ScoringParams())
    req = make_log(lines, trig, seed=13, hit_rate=0.01)
    for trace in (False, True):
        eng = Engine(lib, Config.load(overrides={"engine.device": str(dev), "engine.trace": str(trace).lower()}),
                     device=dev)
        for _ in range(5):
            out = eng.analyze_batch_json([req])
        lat = []
        for _ in range(50):
            t = time.perf_counter()
            out = eng.analyze_batch_json([req])
            lat.append(time.perf_counter() - t)
        rec = {"trace": trace, "lines": lines, "p50_ms": round(float(np.median(lat)) * 1e3, 3),
               "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3)}
        if trace:
            rec["stages"] = json.loads(out[0])["metadata"]["stageTimingsMs"]
        print(json.dumps(rec), flush=True)
    eng.profile = False
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if dev.type == "cuda" else [])
    with profile(activities=acts) as prof:
        for _ in range(10):
            eng.analyze_batch_json([req])
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30))


if __name__ == "__main__":
    main()
