"""Device-resident frequency state (frequency.DeviceFrequencyState + csrc/kernels/freq_state.hip):
the sliding window of FrequencyTrackingService.java:41-93 kept in HBM. With a fake clock the
engine's scores must equal the golden model's across window eviction, request after request;
the admin / snapshot API must agree with the host state."""
import json
import random

import numpy as np
import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine
from log_parser_amd.frequency import DeviceFrequencyState, FrequencyState
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


def _run(device, tmp_path):
    p = ScoringParams()
    sets, trig = make_library(30, seed=41)
    lib = CompiledLibrary(sets, p)
    clk = [1_000_000.0]
    clock = lambda: clk[0]  # noqa: E731
    freq = DeviceFrequencyState(lib.freq_ids, p.freq_window_hours, device, clock=clock, capacity=8)
    eng = Engine(lib, Config.load(overrides={"engine.device": str(device)}), device=torch.device(device), freq=freq)
    tracker = golden.FrequencyTracker(p, clock=clock)
    rng = random.Random(4)
    first, lowered = {}, 0
    for req in range(7):
        logs = make_log(600, trig, seed=100 + req % 2, hit_rate=0.3)
        r = eng.analyze(logs)
        g = golden.analyze(logs, sets, p, tracker)
        assert len(r["events"]) == len(g["events"]) > 0
        np.testing.assert_allclose([e["score"] for e in r["events"]], [e["score"] for e in g["events"]], rtol=1e-12)
        sc = [e["score"] for e in r["events"]]
        if req % 2 in first:                                   # same log again: penalised or not
            lowered += sum(a < b for a, b in zip(sc, first[req % 2]))
        first.setdefault(req % 2, sc)
        clk[0] += rng.choice([600.0, 1500.0, 2400.0])       # some requests fall out of the 1 h window
        assert freq.statistics() == {k: v for k, v in tracker.statistics().items() if k in freq.statistics()}
    assert lowered > 0                                         # the carry mattered
    assert freq.cap > 8                                        # the ring grew on the device
    # snapshot / restore round trip reproduces the window
    path = str(tmp_path / "freq.json")
    freq.snapshot(path)
    fresh = DeviceFrequencyState(lib.freq_ids, p.freq_window_hours, device, clock=clock)
    fresh.restore(path)
    assert fresh.statistics() == freq.statistics()
    host = FrequencyState(p.freq_window_hours, clock=clock)
    host.restore(path)
    assert host.statistics() == freq.statistics()
    pid = next(iter(freq.statistics()))
    freq.reset(pid)
    assert freq.get_pattern_frequency(pid)["currentCount"] == 0
    freq.reset_all()
    assert freq.statistics() == {}


def test_device_frequency_state_matches_golden_cpu(tmp_path):
    _run("cpu", tmp_path)


@pytest.mark.gpu
def test_device_frequency_state_matches_golden_gpu(gpu_device, tmp_path):
    _run(str(gpu_device), tmp_path)


def test_gpu_engine_defaults_to_device_state(monkeypatch):
    p = ScoringParams()
    sets, _ = make_library(10, seed=2)
    lib = CompiledLibrary(sets, p)
    e = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    assert isinstance(e.freq, FrequencyState)                 # CPU engine: host state
    assert Config.load()["engine.frequency.device-resident"] is True


def test_to_host_state_copies_the_window():
    """The CPU fallback's host copy of a device window (here the CPU twin of the device state)."""
    from log_parser_amd.frequency import DeviceFrequencyState, MirroredFrequencyState
    import numpy as np
    ids = [f"p{i}" for i in range(300)]
    d = DeviceFrequencyState(ids, 1, "cpu", clock=lambda: 1000.0)
    c = np.zeros(300, np.int64)
    c[[0, 7, 299]] = [3, 1, 5]
    d.record_counts(ids, c)
    h = d.to_host_state()
    assert h.statistics() == d.statistics() == {"p0": 3, "p7": 1, "p299": 5}
    m = MirroredFrequencyState(d)
    m.record_counts(ids, c)
    assert m.statistics() == d.statistics() == {"p0": 6, "p7": 2, "p299": 10}
