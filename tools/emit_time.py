import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, torch, sys
from log_parser_amd.engine import Engine
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_log, realistic_library
sets, trig = realistic_library(1000, seed=7)
eng = Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))  # (the host emitter: device-independent)
logs = make_log(10_000, trig, seed=13, hit_rate=0.01)
job = eng.pack_batch([logs])
eng.device_batch(job)
for rep in range(3):
    ts = []
    for _ in range(300):
        t0 = time.perf_counter(); out = eng.emit_batch(job); ts.append(time.perf_counter() - t0)
    ts.sort(); print("emit us median", round(ts[len(ts)//2] * 1e6, 1), "p10", round(ts[len(ts)//10]*1e6, 1))
