import cProfile, pstats, sys, io
sys.path.insert(0, ".")
import torch
from log_parser_amd.engine import Engine
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_log, realistic_library
sets, trig = realistic_library(1000, seed=7)
eng = Engine(CompiledLibrary(sets, ScoringParams()), Config.load(overrides={"engine.device": "cuda:0"}), device=torch.device("cuda", 0))
logs = make_log(10000, trig, seed=13, hit_rate=0.01).encode()
for _ in range(20): eng.analyze_batch_json([logs])
pr = cProfile.Profile()
pr.enable()
for _ in range(200): eng.analyze_batch_json([logs])
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
print(s.getvalue())
