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


def test_bulk_context_features_dense_windows_equal_host_twins(gpu_device):
    """Dense context windows over 300k lines: every k_feat_cov workgroup holds more covered lines
    than lanes (512 lines per workgroup at this size). Lines of different lengths, feature words,
    stack frames and final terminators (U+0085, U+2028, a lone '\\r')."""
    pats = [{"id": "hb", "name": "heartbeat", "severity": "LOW",
             "primary_pattern": {"regex": "heartbeat", "confidence": 0.5},
             "context_extraction": {"lines_before": 3, "lines_after": 2}}]
    lib = CompiledLibrary([PatternSet.model_validate({"metadata": {"library_id": "ctx", "version": "1"},
                                                      "patterns": pats})], ScoringParams())
    tails = ["", " ERROR disk", " warn: slow", " java.lang.IllegalStateException: x", " Error", "\u0085",
             "\u2028", "\r", " FATAL" + " pad" * 40, " ok" * 3]
    lines = []
    for i in range(300_000):
        if i % 11 == 5:
            lines.append(f"\tat com.x.Y{i % 13}.run(Y.java:{i % 97})")
        else:
            lines.append(f"{i % 60:02d} node-{i % 7} heartbeat{tails[(i * 7) % len(tails)]}" + "x" * (i % 23))
    d, c = _run_both(lib, "\n".join(lines).encode(), gpu_device)
    assert d["line"].numel() > 250_000
    _assert_same(d, c)


def test_deferred_dp_step_overflow_reruns_and_records_once(gpu_device):
    """A DP step reads no counts until its end (device-count events, overflow flag in the payload).
    With every capacity far too small the first attempt overflows: its frequency record is vetoed
    on the device, the step re-runs with learned capacities, and the result and the window equal
    a plain engine run's."""
    from log_parser_amd.parallel.dp import ShardedAnalyzer
    sets, trig = realistic_library(200, seed=41)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(60_000, trig, seed=42, hit_rate=0.05).encode()
    e1, e2 = _eng(lib, gpu_device), _eng(lib, gpu_device)
    t = _text(gpu_device, data)
    ls, ll = K.split_lines(t, len(data))
    e1.arena.rate = {k: 1e-6 for k in e1.arena.rate}
    out = ShardedAnalyzer(e1).step(t, len(data), ls, ll, 0, 0, topk=10, pack_events=True)
    ref = e2.run(t, len(data), ls, ll, Segments.single(ls.numel(), gpu_device), e2.freq_carry())
    ne = ref.ev_line.numel()
    assert ne > 1000 and e1.arena.last["events"] == ne
    assert torch.equal(out.result.ev_line, ref.ev_line) and torch.equal(out.result.ev_pat, ref.ev_pat)
    torch.testing.assert_close(out.result.score, ref.score, rtol=0, atol=0)
    assert out.events_packed.numel() == 20 * ne
    e2.commit_frequency(ref.freq_counts)
    assert e1.freq.statistics() == e2.freq.statistics()
    # a second step runs within the learned capacities: no re-run, same window evolution
    out2 = ShardedAnalyzer(e1).step(t, len(data), ls, ll, 0, 0, topk=10)
    assert torch.equal(out2.result.ev_line, ref.ev_line)


def _fused_split(eng, t, n):
    box = []
    ls, ll = K.split_lines(t, n, fused=lambda nlp: box.append(eng.prefilter_early(t, n, nlp)))
    return ls, ll, box[0]


@pytest.mark.parametrize("size_mb", [1, 40])      # 40 MB: the 4-units-per-lane (bulk) prefilter variant
def test_fused_line_index_equals_plain(gpu_device, size_mb):
    """The line index's first pass folded into the literal prefilter (k_prefilter<..., NLF>) gives the
    same line starts / lengths / block index as k_nl_count, on mixed "\\n" / "\\r\\n" text with
    separators straddling 16-byte units and 16 KiB tiles, lone '\\r's, trailing empty lines and an
    unterminated last line; and the prefilter's own output is unchanged."""
    import random
    sets, trig = realistic_library(100, seed=51)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = _eng(lib, gpu_device)
    rng = random.Random(size_mb)
    base = make_log(20_000, trig, seed=52, hit_rate=0.05).split("\n")
    parts, total = [], 0
    while total < size_mb << 20:
        ln = rng.choice(base)
        if rng.random() < 0.05:
            ln += "\r"                                     # a lone '\r' before the separator
        sep = "\r\n" if rng.random() < 0.3 else "\n"
        if rng.random() < 0.01:
            ln = ln[: rng.randint(0, 20)]
        parts.append(ln + sep)
        total += len(ln) + len(sep)
    data = "".join(parts)
    # separators exactly at unit / tile boundaries
    for edge in (16 * 1024 - 1, 16 * 1024, 2 * 16 * 1024 - 2, 15, 16, 31):
        if edge + 2 < len(data):
            data = data[:edge] + "\r\n" + data[edge + 2:]
    data = data.rstrip("\n") + "tail without newline\n\n\n"
    raw = data.encode()
    t = _text(gpu_device, raw)
    n = len(raw)
    ls1, ll1 = K.split_lines(t, n)
    ls2, ll2, early = _fused_split(eng, t, n)
    assert torch.equal(ls1, ls2) and torch.equal(ll1, ll2)
    assert torch.equal(ls1._lp_blk[0], ls2._lp_blk[0])
    plain = K.EarlyPrefilter(t, n, eng.tabs, eng.arena, eng.pf_grid)
    c1, c2 = int(plain.cnt[0]), int(early.cnt[0])
    assert c1 == c2 and c1 <= plain.cap
    assert torch.equal(torch.sort(plain.gh[:c1]).values, torch.sort(early.gh[:c2]).values)
