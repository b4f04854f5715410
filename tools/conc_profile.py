"""Where does a continuous-batching batch spend its time? One 2048-request mixed batch through
Engine.analyze_batch_json: stage timings (engine.trace) + cProfile of the host side."""
import cProfile
import io
import json
import pstats
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
    n_req = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    sets, trig = make_library(1000, seed=7)
    lib = CompiledLibrary(sets, ScoringParams())
    rng = np.random.default_rng(0)
    sizes = rng.choice([20, 100, 500, 2000, 10000], size=n_req, p=[0.3, 0.3, 0.2, 0.15, 0.05])
    pool = {s: [make_log(int(s), trig, seed=int(s) + k, hit_rate=0.01) for k in range(4)] for s in set(sizes.tolist())}
    reqs = [pool[int(s)][i % 4] for i, s in enumerate(sizes)]
    for trace in (False, True):
        eng = Engine(lib, Config.load(overrides={"engine.device": str(dev), "engine.trace": str(trace).lower()}),
                     device=dev)
        for _ in range(3):
            eng.analyze_batch_json(reqs)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            outs = eng.analyze_batch_json(reqs)
        dt = (time.perf_counter() - t0) / reps
        rec = {"trace": trace, "requests": n_req, "lines": int(sizes.sum()), "batch_ms": round(dt * 1e3, 3),
               "req_per_s": round(n_req / dt, 1), "bytes": sum(len(r) for r in reqs)}
        if trace:
            rec["stages"] = json.loads(outs[0])["metadata"]["stageTimingsMs"]
        print(json.dumps(rec), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    eng.analyze_batch_json(reqs)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
