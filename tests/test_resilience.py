"""Failure handling: device-failure fallback, stream checkpoint/resume, DP fault detection."""
import json

import numpy as np
import torch
from fastapi.testclient import TestClient

from log_parser_amd import golden
from log_parser_amd.engine import Engine
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.serve.app import create_app
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


def test_device_failure_falls_back_to_cpu_backend():
    sets, trig = make_library(20, seed=61)
    lib = CompiledLibrary(sets, ScoringParams())
    cfg = Config.load(overrides={"engine.device": "cpu", "engine.fault-inject-every": "2",
                                 "engine.batch.max-wait-ms": "0"})
    eng = Engine(lib, cfg, device=torch.device("cpu"))
    fz = golden.FrequencyTracker(ScoringParams())
    with TestClient(create_app(cfg, engine=eng)) as c:
        for i in range(4):      # batches 2 and 4 fail on the "device" and are served by the fallback
            logs = make_log(300, trig, seed=70 + i, hit_rate=0.06)
            r = c.post("/parse", json={"pod": {}, "logs": logs})
            assert r.status_code == 200
            g = golden.analyze(logs, sets, ScoringParams(), fz)
            assert [e["lineNumber"] for e in r.json()["events"]] == [e["lineNumber"] for e in g["events"]]
            assert r.json()["summary"] == g["summary"]    # frequency state shared with the fallback
        assert "lp_device_failures_total 2" in c.get("/metrics").text


def _serve_with_faults(device, overrides, n=5, params=None):
    params = params or ScoringParams(freq_threshold=1.0)
    sets, trig = make_library(20, seed=62)
    lib = CompiledLibrary(sets, params)
    cfg = Config.load(overrides={"engine.device": str(device), "engine.batch.max-wait-ms": "0", **overrides})
    eng = Engine(lib, cfg, device=device)
    fz = golden.FrequencyTracker(params)
    with TestClient(create_app(cfg, engine=eng)) as c:
        for i in range(n):
            logs = make_log(300, trig, seed=170 + i, hit_rate=0.08)
            r = c.post("/parse", json={"pod": {}, "logs": logs})
            assert r.status_code == 200
            g = golden.analyze(logs, sets, params, fz)
            assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in r.json()["events"]] == \
                [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
            np.testing.assert_allclose([e["score"] for e in r.json()["events"]], [e["score"] for e in g["events"]],
                                       rtol=1e-12)
        return c.get("/metrics").text, eng.freq.statistics()


def test_failure_after_record_is_not_recorded_twice():
    """A batch that fails AFTER its counts entered the window is served by the fallback without
    a second record: later batches see exactly the reference's frequency penalties."""
    metrics, stats = _serve_with_faults(torch.device("cpu"), {"engine.fault-inject-after-record": "2"})
    assert "lp_device_failures_total 2" in metrics


def test_stream_checkpoint_resume_is_exact(tmp_path):
    import pytest
    from log_parser_amd.parallel.stream import StreamAnalyzer
    sets, trig = make_library(30, seed=81, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(3000, trig, seed=82, hit_rate=0.08).encode()
    ref = StreamAnalyzer(Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu")),
                         chunk_bytes=8192, topk=10).run(data)
    ck = str(tmp_path / "stream.ckpt.npz")
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    with pytest.raises(RuntimeError, match="injected"):
        StreamAnalyzer(eng, chunk_bytes=8192, topk=10).run(data, checkpoint=ck, fail_after_chunks=5)
    out = StreamAnalyzer(eng, chunk_bytes=8192, topk=10).run(data, checkpoint=ck, resume=ck)
    assert out.chunks == ref.chunks and out.total_lines == ref.total_lines
    for a, b in zip(out.events, ref.events):
        np.testing.assert_array_equal(a, b)
    assert out.summary == ref.summary


import pytest  # noqa: E402


@pytest.mark.gpu
def test_gpu_fallback_uses_host_copy_of_device_window(gpu_device):
    """Device-resident window: the CPU fallback reads a host copy of it (not the GPU) and records
    back; failures before and after the runner's record keep the reference penalties."""
    m1, _ = _serve_with_faults(gpu_device, {"engine.fault-inject-every": "2"})
    assert "lp_device_failures_total 2" in m1
    m2, _ = _serve_with_faults(gpu_device, {"engine.fault-inject-after-record": "2"})
    assert "lp_device_failures_total 2" in m2
