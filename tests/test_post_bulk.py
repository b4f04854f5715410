"""GPU: the bucket-sorted bulk post-match path (csrc/kernels/post_bulk.hip) against the host twins.

Batches here have more candidates / events than the single-workgroup request path holds, so the
device runs the bulk path: regex buckets (split by line block when hot), line-block event buckets
and frequency-key buckets (split by event block when hot). The host twins (std::sort) are the
reference; hits, events, ranks and counts must be identical, scores equal to 1e-14."""
import numpy as np
import pytest
import torch

from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.models.schema import PatternSet
from log_parser_amd.ops import kernels as K
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_log, realistic_library

pytestmark = pytest.mark.gpu


def _eng(lib, dev):
    return Engine(lib, Config.load(overrides={"engine.device": str(dev)}), device=dev)


def _text(dev, data: bytes):
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy())
    return t.to(dev)


def _run_both(lib, data: bytes, gpu):
    outs = []
    for dev in (gpu, torch.device("cpu")):
        e = _eng(lib, dev)
        t = _text(dev, data)
        ls, ll = K.split_lines(t, len(data))
        hits = e.match_hits(t, len(data), ls, ll).cpu()
        res = e.run(t, len(data), ls, ll, Segments.single(ls.numel(), dev), e.freq_carry(), with_factors=True)
        outs.append({"hits": hits, "line": res.ev_line.cpu(), "pat": res.ev_pat.cpu(), "score": res.score.cpu(),
                     "factors": res.factors.cpu(), "freq": res.freq_counts.cpu()})
    return outs


def _assert_same(d, c):
    assert torch.equal(d["hits"], c["hits"])
    assert torch.equal(d["line"], c["line"]) and torch.equal(d["pat"], c["pat"])
    assert torch.equal(d["freq"], c["freq"])
    # the device exp() may differ from the host libm's by an ulp (as in test_gpu.py)
    torch.testing.assert_close(d["factors"], c["factors"], rtol=1e-14, atol=0)
    torch.testing.assert_close(d["score"], c["score"], rtol=1e-14, atol=0)


def test_bulk_path_realistic_library_equals_host_twins(gpu_device):
    sets, trig = realistic_library(400, seed=31)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(120_000, trig, seed=32, hit_rate=0.05, aux_rate=0.02, stack_rate=0.01)
    d, c = _run_both(lib, logs.encode(), gpu_device)
    assert d["hits"].numel() > 4096 and d["line"].numel() > 4096     # beyond the request path's capacity
    _assert_same(d, c)


def _hot_library():
    """A regex that matches every line (hot regex bucket: split into line-block sub-buckets), three
    patterns on it sharing one id (hot frequency key: split into event-block sub-buckets), and a
    literal repeated thousands of times on one line (one (regex, line) with > 4096 candidate copies:
    the tiled LDS sort + global merge passes)."""
    pats = [
        {"id": "hot", "name": "heartbeat a", "severity": "LOW",
         "primary_pattern": {"regex": "heartbeat ok", "confidence": 0.5},
         "context_extraction": {"lines_before": 2, "lines_after": 1}},
        {"id": "hot", "name": "heartbeat b", "severity": "MEDIUM",
         "primary_pattern": {"regex": "heartbeat ok", "confidence": 0.7}},
        {"id": "hot", "name": "heartbeat c", "severity": "HIGH",
         "primary_pattern": {"regex": r"heartbeat\s+ok", "confidence": 0.9},
         "secondary_patterns": [{"regex": "zqxrep", "weight": 0.5, "proximity_window": 50}]},
        {"id": "rep", "name": "repeated token", "severity": "CRITICAL",
         "primary_pattern": {"regex": "zqxrep", "confidence": 0.8}},
    ]
    return [PatternSet.model_validate({"metadata": {"library_id": "hot", "version": "1"}, "patterns": pats})]


def test_bulk_path_hot_buckets_equal_host_twins(gpu_device):
    lib = CompiledLibrary(_hot_library(), ScoringParams())
    lines = [f"2026-10-17T10:00:{i % 60:02d}Z node-{i % 7} heartbeat ok seq={i}" for i in range(60_000)]
    lines[777] = "burst " + "zqxrep " * 6000                      # 6000 copies of one (regex, line)
    lines[30_000] = "zqxrep once"
    d, c = _run_both(lib, "\n".join(lines).encode(), gpu_device)
    assert d["line"].numel() > 3 * 59_000                            # every line, three patterns
    _assert_same(d, c)
