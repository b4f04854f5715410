"""GPU (MI355X) tests: every HIP kernel against its host twin and the pure-Python golden model."""
import math
import os
import random

import numpy as np
import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log

pytestmark = pytest.mark.gpu


def _eng(lib, dev):
    return Engine(lib, Config.load(overrides={"engine.device": str(dev)}), device=dev)


def test_native_extension_is_in_tree_and_hip(gpu_device):
    import sys
    from log_parser_amd.native import load
    m = load()
    assert os.path.dirname(os.path.abspath(m.__file__)).endswith("log_parser_amd")
    assert "log_parser_amd._lpnative" in sys.modules


def _text(dev, data: bytes):
    size = K.padded_len(len(data))
    t = torch.zeros(size, dtype=torch.uint8)
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    return t.to(dev), t


def _tile_edge_texts():
    T = K.NL_TILE
    yield from ["", "\n", "\n\n", "\r\n", "a", "a\n", "\r", "\r\r\n", "a\r\n\r\n", "\n\na"]
    yield "x" * (3 * T + 5)                                     # one line over four tiles
    yield "x" * (T - 1) + "\n" + "y" * 10                        # '\n' on a tile's last byte
    yield "x" * T + "\n" + "y"                                   # '\n' on a tile's first byte
    yield "x" * (T - 1) + "\r\nz\n"                              # CRLF across a tile boundary
    yield "x" * (2 * T - 1) + "\r" + "\n" * 3                     # ... then trailing empty lines
    yield "x" * (4 * T - 1) + "\r\nz\n" + "w" * (4 * T)            # same at the 64 KiB look-back tiles
    yield "x" * (4 * T) + "\n" + "y"
    yield "".join(f"line {i} with some words in it\n" for i in range(200000))   # ~400 tiles: look-back
    yield "\n" * (5 * T)                                        # only empty lines: none kept
    yield "ab\n" * (4 * T)                                      # above the capacity guess: re-run
    for n in (5, 6, 7, 9):                                       # tile counts off the 4-tile workgroups
        yield "".join(f"r{i} \r\n" if i % 7 == 0 else f"row {i}\n" for i in range(n * T // 9)) + "x" * 3
    yield "a\rb\n" * (T // 2) + "tail"                            # stray '\r's: flagged tiles, no CRLF
    yield "x" * (T + 7) + "\n" + "y" * 3                          # partial 16-byte piece at the end


def test_line_index_tile_edges(gpu_device):
    """Line index (k_nl_count masks, k_nl_lines over 4-tile workgroups): tile boundaries, CR across
    a boundary, stray CRs, all-empty / no-newline texts, many tiles, tile counts that are not a
    multiple of 4, capacity re-run -- equal to Java split."""
    for s in _tile_edge_texts():
        data = s.encode()
        td, _ = _text(gpu_device, data)
        ls_d, ll_d = K.split_lines(td, len(data))
        ref = golden.split_lines(s)
        assert ls_d.numel() == len(ref), (len(s), s[:20])
        got = [data[a:a + b].decode() for a, b in zip(ls_d.cpu().tolist(), ll_d.cpu().tolist())]
        assert got == ref, (len(s), s[:20])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_line_index_matches_java_split(gpu_device, seed):
    rng = random.Random(seed)
    parts = []
    for _ in range(rng.randint(0, 50000)):
        parts.append(rng.choice(["", "a", "xyz", "\r", "é", "line with words"]) * rng.randint(0, 5))
        parts.append(rng.choice(["\n", "\r\n", "\n", "\n"]))
    s = "".join(parts) + rng.choice(["", "\n", "\n\n\r\n", "tail"])
    data = s.encode()
    td, tc = _text(gpu_device, data)
    ls_d, ll_d = K.split_lines(td, len(data))
    ls_c, ll_c = K.split_lines(tc, len(data))
    assert torch.equal(ls_d.cpu(), ls_c) and torch.equal(ll_d.cpu(), ll_c)
    ref = golden.split_lines(s)
    assert ls_c.numel() == len(ref)
    got = [data[a:a + b].decode() for a, b in zip(ls_c.tolist(), ll_c.tolist())]
    assert got == ref


@pytest.mark.parametrize("mb", [37, 301])
def test_line_index_large_tile_scan(gpu_device, mb):
    """Many tiles (2.4k / 19k, an odd count): every thread of the one-workgroup tile scan
    (k_tile_scan) sums a run of several counts, with a scalar tail -- equal to the host index."""
    rng = np.random.default_rng(mb)
    n = mb * (1 << 20) + 12345
    data = rng.integers(32, 127, size=n, dtype=np.uint8)
    nl = rng.random(n) < 1 / 90                                  # ~90-byte lines, some empty
    data[nl] = 10
    data[rng.random(n) < 1 / 5000] = 13
    b = data.tobytes()
    td, tc = _text(gpu_device, b)
    ls_d, ll_d = K.split_lines(td, len(b))
    ls_c, ll_c = K.split_lines(tc, len(b))
    assert ls_d.numel() == ls_c.numel() > 1000
    assert torch.equal(ls_d.cpu(), ls_c) and torch.equal(ll_d.cpu(), ll_c)


@pytest.mark.parametrize("n_pat,seed", [(64, 1), (300, 5)])
def test_hits_gpu_equal_cpu(gpu_device, n_pat, seed):
    sets, trig = make_library(n_pat, seed=seed)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(20000, trig, seed=seed + 1, hit_rate=0.05, crlf_rate=0.1)
    data = logs.encode()
    ed, ec = _eng(lib, gpu_device), _eng(lib, torch.device("cpu"))
    td, tc = _text(gpu_device, data)
    ls_d, ll_d = K.split_lines(td, len(data))
    ls_c, ll_c = K.split_lines(tc, len(data))
    hd = ed.match_hits(td, len(data), ls_d, ll_d)
    hc = ec.match_hits(tc, len(data), ls_c, ll_c)
    assert hd.numel() > 100
    assert torch.equal(hd.cpu(), hc)


@pytest.mark.parametrize("seed", [3, 4])
def test_engine_gpu_matches_golden(gpu_device, seed):
    p = ScoringParams()
    sets, trig = make_library(60, seed=seed)
    lib = CompiledLibrary(sets, p)
    logs = make_log(3000, trig, seed=seed + 10, hit_rate=0.06)
    eng = _eng(lib, gpu_device)
    for rep in range(2):   # second pass exercises the persistent frequency carry
        r = eng.analyze(logs)
        g = golden.analyze(logs, sets, p, _FREQ.setdefault(seed, golden.FrequencyTracker(p)))
        assert len(r["events"]) == len(g["events"]) > 0
        for a, b in zip(r["events"], g["events"]):
            assert a["lineNumber"] == b["lineNumber"]
            assert a["matchedPattern"]["id"] == b["matchedPattern"]["id"]
            assert a["context"] == b["context"]
            assert math.isclose(a["score"], b["score"], rel_tol=1e-12), (a["score"], b["score"])
        assert r["summary"] == g["summary"]


_FREQ = {}


def test_score_factors_gpu_equal_cpu(gpu_device):
    sets, trig = make_library(80, seed=9)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(5000, trig, seed=19, hit_rate=0.05)
    data = logs.encode()
    outs = []
    for dev in (gpu_device, torch.device("cpu")):
        e = _eng(lib, dev)
        t, _ = _text(dev, data)
        ls, ll = K.split_lines(t, len(data))
        res = e.run(t, len(data), ls, ll, Segments.single(ls.numel(), dev), e.freq_carry(), with_factors=True)
        outs.append((res.score.cpu(), res.factors.cpu(), res.ev_line.cpu(), res.ev_pat.cpu()))
    (s1, f1, l1, p1), (s2, f2, l2, p2) = outs
    assert torch.equal(l1, l2) and torch.equal(p1, p2)
    torch.testing.assert_close(f1, f2, rtol=1e-14, atol=0)
    torch.testing.assert_close(s1, s2, rtol=1e-14, atol=0)


def test_sharded_single_rank_equals_engine(gpu_device):
    from log_parser_amd.parallel.dp import ShardedAnalyzer
    sets, trig = make_library(50, seed=21)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(4000, trig, seed=22, hit_rate=0.05)
    data = logs.encode()
    e1, e2 = _eng(lib, gpu_device), _eng(lib, gpu_device)
    t, _ = _text(gpu_device, data)
    ls, ll = K.split_lines(t, len(data))
    out = ShardedAnalyzer(e1).step(t, len(data), ls, ll, 0, 0, topk=10)
    ref = e2.run(t, len(data), ls, ll, Segments.single(ls.numel(), gpu_device), e2.freq_carry())
    assert torch.equal(out.result.ev_line, ref.ev_line)
    torch.testing.assert_close(out.result.score, ref.score, rtol=0, atol=0)
    top = torch.topk(ref.score, 10).values
    torch.testing.assert_close(out.topk_score, top)


def test_run_document_equals_run_and_records(gpu_device):
    """Engine.run_document (config 2's resident path: line index + early prefilter, deferred
    counts, one read at the end) equals split_lines + run, twice in a row (the second document
    sees the first one's frequency record in both engines)."""
    sets, trig = make_library(80, seed=31)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(6000, trig, seed=32, hit_rate=0.05).encode()
    e1, e2 = _eng(lib, gpu_device), _eng(lib, gpu_device)
    t, _ = _text(gpu_device, data)
    for _ in range(2):
        doc = e1.run_document(t, len(data), with_factors=True)
        ls, ll = K.split_lines(t, len(data))
        ref = e2.run(t, len(data), ls, ll, Segments.single(ls.numel(), gpu_device), e2.freq_carry(), with_factors=True)
        e2.commit_frequency(ref.freq_counts)
        assert doc.ev_line.numel() == ref.ev_line.numel() > 0
        assert torch.equal(doc.ev_line, ref.ev_line) and torch.equal(doc.ev_pat, ref.ev_pat)
        assert torch.equal(doc.hit_keys, ref.hit_keys)
        torch.testing.assert_close(doc.score, ref.score, rtol=0, atol=0)
        torch.testing.assert_close(doc.factors, ref.factors, rtol=0, atol=0)
        assert torch.equal(doc.freq_counts, ref.freq_counts)


def test_run_document_overflow_rerun_records_once(gpu_device):
    """run_document queues the frequency record before its count read, gated on the device by the
    buffer capacities: a first attempt that overflows (capacities forced tiny) records nothing and
    the re-run records once -- the next document's scores see exactly one record."""
    sets, trig = make_library(80, seed=33)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(6000, trig, seed=34, hit_rate=0.2).encode()
    e1, e2 = _eng(lib, gpu_device), _eng(lib, gpu_device)
    t, _ = _text(gpu_device, data)
    for _ in range(3):
        e1.arena.rate = {k: 1e-4 for k in e1.arena.rate}   # every document overflows its first attempt
        doc = e1.run_document(t, len(data))
        ls, ll = K.split_lines(t, len(data))
        ref = e2.run(t, len(data), ls, ll, Segments.single(ls.numel(), gpu_device), e2.freq_carry())
        e2.commit_frequency(ref.freq_counts)
        assert doc.ev_line.numel() == ref.ev_line.numel() > 600
        torch.testing.assert_close(doc.score, ref.score, rtol=0, atol=0)
        assert torch.equal(e1.freq_carry(), e2.freq_carry())


def _strip(o):
    o = dict(o)
    o.pop("analysisId")
    o["metadata"] = {k: v for k, v in o["metadata"].items() if k not in ("processingTimeMs", "analyzedAt")}
    return o


def test_batch_edge_cases_gpu_equal_cpu_and_golden(gpu_device):
    """One device batch of awkward documents (empty, newline-only, CRLF, multi-byte UTF-8, a
    200 KB line, event windows at document edges) with the shipped example pattern library:
    GPU responses == CPU-backend responses == golden model."""
    import json
    import os
    from log_parser_amd.models.library import load_pattern_directory
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sets = load_pattern_directory(os.path.join(root, "patterns", "examples"))
    p = ScoringParams()
    lib = CompiledLibrary(sets, p)
    oom = "java.lang.OutOfMemoryError: Java heap space"
    docs = ["", "\n", "\n\n\r\n", oom, oom + "\r\n", "é" * 1000 + " " + oom + "\n\tat com.x.Y(Z.java:1)\n",
            ("INFO ok\r\n" * 50) + oom + "\r\n" + ("WARN later\r\n" * 3),
            "x" * 200_000 + " OutOfMemoryError\n" + "ERROR Exception in thread main\n" * 5,
            "\n".join(["CrashLoopBackOff", "Back-off restarting failed container", "OOMKilled"] * 30)]
    outs = {}
    for dev in (gpu_device, torch.device("cpu")):
        eng = _eng(lib, dev)
        outs["gpu" if dev is gpu_device else "cpu"] = [_strip(json.loads(o)) for o in eng.analyze_batch_json(docs)]
    assert outs["gpu"] == outs["cpu"]
    tracker = golden.FrequencyTracker(p)
    for d, o in zip(docs, outs["gpu"]):
        g = golden.analyze(d, sets, p, tracker)
        assert o["summary"] == g["summary"]
        assert [(e["lineNumber"], e["matchedPattern"]["id"], e["context"]) for e in o["events"]] == \
               [(e["lineNumber"], e["matchedPattern"]["id"], e["context"]) for e in g["events"]]
        for a, b in zip(o["events"], g["events"]):
            assert math.isclose(a["score"], b["score"], rel_tol=1e-12)
    assert sum(len(o["events"]) for o in outs["gpu"]) > 10


@pytest.mark.parametrize("seed", [7, 8])
def test_native_runner_equals_python_orchestration(gpu_device, seed):
    """csrc/runtime/request.cpp runs the same kernels as Engine.prepare / finish: over a sequence
    of batches (the device frequency window evolving through them, one batch large enough to
    overflow the first matcher capacities) the responses are identical with the runner on and
    off, and the runner path really ran."""
    import json
    sets, trig = make_library(300, seed=seed)
    lib = CompiledLibrary(sets, ScoringParams())
    batches = [[make_log(3000, trig, seed=seed * 10 + i, hit_rate=0.05) for i in range(3)],
               [make_log(20_000, trig, seed=seed * 10 + 5, hit_rate=0.3)],
               [make_log(500, trig, seed=seed * 10 + 6, hit_rate=0.02), "", "\n"]]
    outs = {}
    for on in (True, False):
        cfg = Config.load(overrides={"engine.device": str(gpu_device), "engine.native-runner": on})
        eng = Engine(lib, cfg, device=gpu_device)
        outs[on] = [[_strip(json.loads(o)) for o in eng.analyze_batch_json(b)] for b in batches]
        assert (eng._runner is not None and eng._runner is not False) == on
    assert outs[True] == outs[False]
    assert sum(len(o["events"]) for b in outs[True] for o in b) > 100


def test_native_runner_device_counts_equals_host_counts(gpu_device):
    """The runner's device-count mode (no mid-batch host read, frequency record gated on the
    capacities) gives the same responses as its host-count mode, including a batch whose matcher
    counts overflow the first capacities (gate closed, re-run)."""
    import json
    sets, trig = make_library(300, seed=9)
    lib = CompiledLibrary(sets, ScoringParams())
    batches = [[make_log(2000, trig, seed=90 + i, hit_rate=0.05)] for i in range(3)] + \
              [[make_log(8000, trig, seed=95, hit_rate=0.4)], [make_log(1000, trig, seed=96, hit_rate=0.05)]]
    outs = {}
    for dc in (True, False):
        cfg = Config.load(overrides={"engine.device": str(gpu_device), "engine.runner-device-counts": dc})
        eng = Engine(lib, cfg, device=gpu_device)
        outs[dc] = [[_strip(json.loads(o)) for o in eng.analyze_batch_json(b)] for b in batches]
    assert outs[True] == outs[False]


def test_native_runner_fetch_publish_equal_orchestration(gpu_device):
    """The runner's k_fetch (inputs read from the pinned stage by a kernel) + k_publish (counters and
    compacted results written into pinned host memory) give the same responses as the Python
    orchestration (engine.native-runner=false), over batches of several documents, an empty one
    and a stage too small for the single-copy layout on its first use."""
    import json
    sets, trig = make_library(200, seed=12)
    lib = CompiledLibrary(sets, ScoringParams())
    batches = [[make_log(3000, trig, seed=120, hit_rate=0.05)],
               [make_log(500, trig, seed=121 + i, hit_rate=0.1) for i in range(4)],
               [""], [make_log(12000, trig, seed=125, hit_rate=0.02)]]
    outs = {}
    for native in (True, False):
        eng = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device), "engine.native-runner": native}),
                     device=gpu_device)
        outs[native] = [[_strip(json.loads(o)) for o in eng.analyze_batch_json(b)] for b in batches]
        assert (eng._runner not in (None, False)) == native
    assert outs[True] == outs[False]
    assert sum(len(o["events"]) for b in outs[True] for o in b) > 50
