"""Chunked streaming (parallel/stream.py) == single-pass analysis of the whole log."""
import numpy as np
import pytest
import torch

from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.parallel.stream import RepeatBuffer, StreamAnalyzer
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


def _eng(lib, dev="cpu"):
    return Engine(lib, Config.load(overrides={"engine.device": dev}), device=torch.device(dev))


@pytest.mark.parametrize("chunk,crlf", [(4096, 0.0), (20000, 0.3), (1 << 20, 0.0)])
def test_stream_equals_single_pass(chunk, crlf):
    sets, trig = make_library(40, seed=41, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(2500, trig, seed=42, hit_rate=0.08, crlf_rate=crlf) + "\n\n\r\n"
    data = logs.encode()
    e1 = _eng(lib)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    ref = e1.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), e1.freq_carry())
    e2 = _eng(lib)
    out = StreamAnalyzer(e2, chunk_bytes=chunk, topk=7).run(data)
    assert out.total_lines == ls.numel()
    if chunk < len(data):
        assert out.chunks > 1
    gl, pat, score = out.events
    np.testing.assert_array_equal(gl, ref.ev_line.numpy())
    np.testing.assert_array_equal(pat, ref.ev_pat.numpy())
    np.testing.assert_allclose(score, ref.score.numpy(), rtol=1e-15, atol=0)
    np.testing.assert_allclose(out.topk_score, np.sort(ref.score.numpy())[::-1][:7], rtol=1e-15)
    assert out.summary == e1.summary(ref.ev_pat.numpy())
    e1.commit_frequency(ref.freq_counts)   # frequency state advanced identically
    assert e1.freq.statistics() == e2.freq.statistics()


def test_stream_edge_inputs():
    sets, trig = make_library(5, seed=1)
    lib = CompiledLibrary(sets, ScoringParams())
    for s, n in [(b"", 1), (b"\n\n", 0), (b"abc", 1), (b"a\n\nb\n\n", 3), (b"a\r\r\n", 1)]:
        assert StreamAnalyzer(_eng(lib), chunk_bytes=2).run(s).total_lines == n, s


def test_repeat_buffer():
    blk = b"ab\ncd\n\nxyz\n"
    rb = RepeatBuffer(blk, 100)
    full = (blk * 20)[:100]
    assert rb[3:57] == full[3:57] and len(rb) == 100 and rb[5] == full[5]
    for st in range(0, 100, 7):
        assert rb.find(b"\n", st) == full.find(b"\n", st)
        assert rb.rfind(b"\n", 0, st) == full.rfind(b"\n", 0, st)


def _dense():
    sets, trig = make_library(40, seed=43, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(4000, trig, seed=44, hit_rate=0.3).encode()      # dense matches
    return lib, data


def test_bounded_topk_mode_equals_full(monkeypatch):
    """keep_events=False keeps only events that can still reach the top-k (bounds from the
    chronological factor's min / max): same top-k, summary and event count as keeping all."""
    lib, data = _dense()
    full = StreamAnalyzer(_eng(lib), chunk_bytes=8192, topk=9).run(data)
    monkeypatch.setattr(StreamAnalyzer, "PRUNE_AT", 64)           # prune after (almost) every chunk
    sa = StreamAnalyzer(_eng(lib), chunk_bytes=8192, topk=9, keep_events=False)
    kept = []
    orig = StreamAnalyzer._prune

    def spy(self, *a):
        out = orig(self, *a)
        kept.append(out[0][0].numel())
        return out
    monkeypatch.setattr(StreamAnalyzer, "_prune", spy)
    b = sa.run(data)
    assert kept and max(kept) < full.n_events // 2               # memory stays bounded
    assert b.n_events == full.n_events and b.summary == full.summary and b.events is None
    np.testing.assert_array_equal(b.topk_line, full.topk_line)
    np.testing.assert_array_equal(b.topk_pat, full.topk_pat)
    np.testing.assert_allclose(b.topk_score, full.topk_score, rtol=1e-15, atol=0)


def test_resident_log_reanalysis_equals_stream():
    """A log loaded into (device) memory once is re-analysed by two libraries without restaging,
    each equal to a host stream of the same bytes."""
    from log_parser_amd.parallel.stream import ResidentLog
    lib, data = _dense()
    sets2, _ = make_library(30, seed=45)
    lib2 = CompiledLibrary(sets2, ScoringParams())
    big = lib if lib.halo >= lib2.halo else lib2
    res = ResidentLog.load(data, _eng(big), chunk_bytes=8192)
    assert len(res.chunks) > 3 and res.device_bytes >= len(data)
    for L in (lib, lib2):
        a = StreamAnalyzer(_eng(L), chunk_bytes=8192, topk=5).run(res)
        b = StreamAnalyzer(_eng(L), chunk_bytes=8192, topk=5).run(data)
        assert a.total_lines == b.total_lines and a.summary == b.summary
        for x, y in zip(a.events, b.events):
            np.testing.assert_array_equal(x, y)


def test_auto_chunk_bytes_cpu():
    from log_parser_amd.parallel.stream import CHUNK_MIN, auto_chunk_bytes
    assert auto_chunk_bytes(torch.device("cpu")) == CHUNK_MIN
    sets, _ = make_library(5, seed=1)
    assert StreamAnalyzer(_eng(CompiledLibrary(sets, ScoringParams()))).chunk_bytes == CHUNK_MIN


def test_auto_chunk_bytes_policy(monkeypatch):
    """HBM cap 1/16 of free memory in [256 MiB, 8 GiB]; a host stream also caps at 1/8 of its length."""
    from log_parser_amd.parallel import stream as S
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d: (280 << 30, 288 << 30))
    dev = torch.device("cuda", 0)
    assert S.auto_chunk_bytes(dev) == S.CHUNK_MAX
    assert S.auto_chunk_bytes(dev, 100 << 30) == S.CHUNK_MAX
    assert S.auto_chunk_bytes(dev, 20 << 30) == (20 << 30) // 8
    assert S.auto_chunk_bytes(dev, 1 << 30) == S.CHUNK_MIN
    assert S.auto_chunk_bytes(dev, 1 << 40) == S.CHUNK_MAX
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d: (1 << 30, 288 << 30))
    assert S.auto_chunk_bytes(dev, 100 << 30) == S.CHUNK_MIN


def test_parse_file_threshold_is_fixed(tmp_path):
    """parse_file streams above engine.stream.threshold-bytes (a fixed size, not the HBM-derived
    chunk), and analyses one whole document below it."""
    from log_parser_amd.api import LogParser
    from log_parser_amd.parallel.stream import StreamResult
    sets, trig = make_library(8, seed=5)
    logs = make_log(300, trig, seed=6, hit_rate=0.1)
    p = tmp_path / "a.log"
    p.write_text(logs)
    size = p.stat().st_size
    big = LogParser(sets, Config.load(overrides={"engine.device": "cpu", "engine.stream.threshold-bytes": size - 1}))
    assert big.stream_threshold() == size - 1
    assert isinstance(big.parse_file(str(p)), StreamResult)
    small = LogParser(sets, Config.load(overrides={"engine.device": "cpu", "engine.stream.threshold-bytes": size}))
    res = small.parse_file(str(p))
    assert isinstance(res, dict) and res["metadata"]["totalLines"] == 300
    assert LogParser(sets, Config.load(overrides={"engine.device": "cpu"})).stream_threshold() == 256 << 20


@pytest.mark.parametrize("m", [0.3, 1.2, 2.5, 4.0])
def test_chrono_bounds_cover_factor(m):
    """_chrono_bounds brackets chrono_factor for any configured max-early-bonus."""
    from log_parser_amd.golden import chronological_factor
    sets, _ = make_library(3, seed=1)
    params = ScoringParams(max_early_bonus=m)
    eng = Engine(CompiledLibrary(sets, params), Config.load(overrides={"engine.device": "cpu"}),
                 device=torch.device("cpu"))
    lo, hi = StreamAnalyzer(eng, chunk_bytes=4096)._chrono_bounds()
    n = 997
    vals = [chronological_factor(i, n, params) for i in range(n)]
    assert lo <= min(vals) and max(vals) <= hi


# ---- one long log streamed over the ranks of a process group (ShardedStreamAnalyzer) ---------
def _sstream_setup(bt=False):
    sets, trig = make_library(40, seed=51, sequence_rate=0.8)
    if bt:
        sets.append(_bt_set())
    lib = CompiledLibrary(sets, ScoringParams())
    data = (make_log(6000, trig, seed=52, hit_rate=0.08, crlf_rate=0.1) + "\n\n").encode()
    return lib, data


def _sstream_worker(rank, world, port, q, dev, chunk, bt=False):
    import os
    import torch.distributed as dist
    from log_parser_amd.parallel.stream import ShardedStreamAnalyzer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lib, data = _sstream_setup(bt)
        eng = _eng(lib, dev)
        outs = []
        for _ in range(2):                    # the second stream sees the first one's window counts
            r = ShardedStreamAnalyzer(eng, chunk_bytes=chunk, topk=9).run(data)
            outs.append((r.total_lines, r.n_events, r.summary, r.topk_score, r.topk_line, r.topk_pat, r.chunks,
                         tuple(np.asarray(x) for x in r.events)))
        q.put((rank, outs, eng.freq.statistics()))
    finally:
        dist.destroy_process_group()


def _run_sstream(world, dev, chunk=9000, bt=False):
    import socket
    import torch.multiprocessing as mp
    lib, data = _sstream_setup(bt)
    e1 = _eng(lib, "cpu")
    refs = [StreamAnalyzer(e1, chunk_bytes=chunk, topk=9).run(data) for _ in range(2)]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sstream_worker, args=(r, world, port, q, dev, chunk, bt)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (o, st)) for r, o, st in (q.get(timeout=600) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, ref in enumerate(refs):
        assert ref.chunks > world                       # several steps of `world` chunks
        gl = np.concatenate([got[r][0][i][7][0] for r in range(world)])
        order = np.argsort(gl, kind="stable")
        pat = np.concatenate([got[r][0][i][7][1] for r in range(world)])[order]
        sc = np.concatenate([got[r][0][i][7][2] for r in range(world)])[order]
        np.testing.assert_array_equal(gl[order], ref.events[0])
        np.testing.assert_array_equal(pat, ref.events[1])
        np.testing.assert_allclose(sc, ref.events[2], rtol=1e-13, atol=0)
        for r in range(world):
            tl, ne, summ, ts, tline, tpat, nch, _ = got[r][0][i]
            assert (tl, ne, summ, nch) == (ref.total_lines, ref.n_events, ref.summary, ref.chunks)
            np.testing.assert_allclose(ts, ref.topk_score, rtol=1e-13)
            np.testing.assert_array_equal(tline, ref.topk_line)
            np.testing.assert_array_equal(tpat, ref.topk_pat)
    for r in range(world):                               # every rank's window recorded the global counts
        assert got[r][1] == e1.freq.statistics()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_stream_equals_single_stream(world):
    """One log streamed over `world` gloo ranks (chunk r of every step on rank r, carries from the
    earlier steps and ranks) equals the single-rank stream event for event, twice in a row."""
    _run_sstream(world, "cpu")


@pytest.mark.gpu
def test_sharded_stream_two_ranks_one_gpu(gpu_device):
    _run_sstream(2, "cuda:0", chunk=1 << 16)


def test_sharded_stream_with_backtracker_regexes():
    """Backtracker regexes in a sharded stream: the side path reads each rank's pinned chunk bytes
    (``host_text``), the same events as the single-rank stream."""
    _run_sstream(2, "cpu", bt=True)


@pytest.mark.gpu
def test_sharded_stream_with_backtracker_regexes_gpu(gpu_device):
    """Same on the GPU: every step's pinned buffer is recycled only after its side-path read, and
    an idle rank's placeholder never enters the pinned pool."""
    _run_sstream(2, "cuda:0", chunk=1 << 14, bt=True)


def _bt_set():
    from log_parser_amd.models.schema import PatternSet
    # (a nested lookaround: plain lookaround clusters compile to DFAs, jregex.cpp LookaroundDfa)
    bt = [r"^(\w*)\1$", r"(\w+)Aux0 \1", r"(?i)fatal (?=\w+Fail(?!ed))"]
    return PatternSet.model_validate({"metadata": {"library_id": "bt"}, "patterns": [
        {"id": f"bt{i}", "name": rx, "severity": "LOW", "primary_pattern": {"regex": rx, "confidence": 0.5}}
        for i, rx in enumerate(bt)]})


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_stream_with_backtracker_regexes_equals_single_pass(dev):
    """Backtracker regexes (host side path on each chunk's pinned bytes, with the chunk line rule:
    no trailing-empty-line removal) stream exactly like one pass -- incl. one that matches the
    empty lines in the middle of the log. On the GPU the chunks are staged and held until their
    prepare ('hold' mode): 10+ chunks through the 3-buffer pinned pool must not deadlock."""
    sets, trig = make_library(20, seed=61, sequence_rate=0.5)
    sets.append(_bt_set())
    lib = CompiledLibrary(sets, ScoringParams())
    assert len(lib.host_plan) == 3
    logs = make_log(2500, trig, seed=62, hit_rate=0.08)
    logs = logs.replace("\n", "\n\n", 40) + "\n\n"
    data = logs.encode()
    e1 = _eng(lib)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    ref = e1.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), e1.freq_carry(),
                 host_text=np.frombuffer(data, np.uint8))
    out = StreamAnalyzer(_eng(lib, dev), chunk_bytes=3000, topk=7).run(data)
    assert out.chunks >= 10
    gl, pat, score = out.events
    np.testing.assert_array_equal(gl, ref.ev_line.numpy())
    np.testing.assert_array_equal(pat, ref.ev_pat.numpy())
    np.testing.assert_allclose(score, ref.score.numpy(), rtol=1e-15 if dev == "cpu" else 1e-12, atol=0)
    assert (pat == lib.patterns.index(next(p for p in lib.patterns if p.id == "bt0"))).sum() >= 40


def test_repeat_buffer_segments():
    rb = RepeatBuffer(b"0123456789", 95)
    segs = rb.segments(7, 33)
    assert sum(t for _, _, t in segs) == 26
    assert b"".join(rb.block[b:b + t] for b, _, t in segs) == rb[7:33]
    assert [o for _, o, _ in segs] == [0, 3, 13, 23]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [1 << 16, 1 << 18])
def test_stream_direct_from_registered_source_equals_staged(gpu_device, chunk):
    """A RepeatBuffer's block is page-locked once and every chunk is copied to the GPU straight
    from it (no staging copy): same events, scores and summary as the staged bytes of that stream."""
    sets, trig = make_library(40, seed=41, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    block = (make_log(1500, trig, seed=45, hit_rate=0.08) + "\n").encode()
    rb = RepeatBuffer(block, 7 * len(block) + 1234)
    assert rb.pinned_block() is not None
    a = StreamAnalyzer(_eng(lib, str(gpu_device)), chunk_bytes=chunk, topk=9).run(rb)
    b = StreamAnalyzer(_eng(lib, str(gpu_device)), chunk_bytes=chunk, topk=9).run(rb[0:len(rb)])
    assert a.total_lines == b.total_lines and a.chunks == b.chunks > 1
    for x, y in zip(a.events, b.events):
        np.testing.assert_array_equal(x, y)
    assert a.summary == b.summary
    np.testing.assert_array_equal(a.topk_score, b.topk_score)
