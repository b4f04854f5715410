"""Data-parallel serving (serve/app.py Batcher with several engines + engine.FrequencyTurn):
batches run concurrently on all engines, yet every response equals the sequential reference
(golden model, one shared frequency tracker, requests in arrival order) -- frequency carries
are read and recorded in batch arrival order."""
import json

import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine, FrequencyTurn, SharedWindowTurn
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.serve.app import Batcher, serve_devices
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.metrics import Metrics
from log_parser_amd.utils.synth import make_library, make_log


def _check(devices, n_req=48, max_requests=3, runner=False):
    # frequent ids and a low threshold so the frequency penalty actually bites across requests
    sets, trig = make_library(25, seed=91)
    params = ScoringParams(freq_threshold=1.0)
    lib = CompiledLibrary(sets, params)
    cfg = Config.load(overrides={"engine.device": str(devices[0])})
    e0 = Engine(lib, cfg, device=devices[0])
    engines = [e0] + [Engine(lib, cfg, device=d, freq=e0.freq) for d in devices[1:]]
    b = Batcher(engines, max_requests, 1 << 30, 0.0, Metrics())
    reqs = [make_log(200 + 37 * (i % 5), trig, seed=900 + i, hit_rate=0.1) for i in range(n_req)]
    futs = [b.submit(r) for r in reqs]
    outs = [json.loads(f.result(timeout=300)) for f in futs]
    b.close()
    if runner:      # every engine served through the native runner on the ONE shared device window
        assert all(e._runner not in (None, False) for e in engines)
        assert all(e.freq is e0.freq and e.freq_on_device for e in engines)
    tracker = golden.FrequencyTracker(params)
    for r, o in zip(reqs, outs):
        g = golden.analyze(r, sets, params, tracker)
        assert o["summary"] == g["summary"]
        assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
               [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
        for a, c in zip(o["events"], g["events"]):
            assert a["score"] == pytest.approx(c["score"], rel=1e-12, abs=0)
    return b


def test_two_cpu_engines_equal_sequential_reference():
    b = _check([torch.device("cpu"), torch.device("cpu")])
    assert b.turn is not None and len(b.engines) == 2


def test_frequency_turn_orders_and_skips():
    t = FrequencyTurn()
    order = []
    import threading
    ths = [threading.Thread(target=lambda s=s: (t.wait(s), order.append(s), t.done(s))) for s in (3, 1, 2)]
    for th in ths:
        th.start()
    t.done(0)                                   # e.g. batch 0 failed: releases its slot
    for th in ths:
        th.join(timeout=10)
    assert order == [1, 2, 3]
    t.done(1)                                   # idempotent
    t.wait(4)


def test_serve_devices_parsing():
    assert serve_devices(Config.load()) == []
    assert serve_devices(Config.load(overrides={"engine.serve-devices": "cpu, cpu"})) == [torch.device("cpu")] * 2


@pytest.mark.gpu
def test_two_engines_on_one_gpu_equal_sequential_reference(gpu_device):
    """Two engines (own HIP streams) on the one test GPU stand in for one engine per GPU: both run
    the native request runner on one shared device-resident window (SharedWindowTurn)."""
    _check([gpu_device, gpu_device], runner=True)


@pytest.mark.gpu
def test_four_engines_shared_window_service(gpu_device):
    """engine.serve-devices=cuda:0 x4 through the Service: identical to sequential serving."""
    from log_parser_amd.serve.app import Service
    sets, trig = make_library(25, seed=93)
    params = ScoringParams(freq_threshold=1.0)
    lib = CompiledLibrary(sets, params)
    dev = str(gpu_device)
    cfg = Config.load(overrides={"engine.device": dev, "engine.serve-devices": ",".join([dev] * 4),
                                 "scoring.frequency.threshold": "1.0", "engine.batch.max-requests": "3"})
    svc = Service(cfg, engine=Engine(lib, cfg, device=gpu_device))
    b = svc.batcher()
    assert len(b.engines) == 4 and isinstance(b.turn, SharedWindowTurn)
    reqs = [make_log(150 + 13 * (i % 7), trig, seed=1900 + i, hit_rate=0.1) for i in range(64)]
    outs = [json.loads(f.result(timeout=300)) for f in [b.submit(r) for r in reqs]]
    svc.close()
    tracker = golden.FrequencyTracker(params)
    for r, o in zip(reqs, outs):
        g = golden.analyze(r, sets, params, tracker)
        assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
               [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
        for a, c in zip(o["events"], g["events"]):
            assert a["score"] == pytest.approx(c["score"], rel=1e-12, abs=0)
    assert sum(e._runner not in (None, False) for e in b.engines) >= 2
