"""Post-match pipeline (csrc/kernels/lp_post.hip): hit CSR, events, frequency ranks, context
coverage/features, fused frequency score input -- host twin against a plain numpy/Python
reference of the same rules, and (GPU) the gfx950 kernels against the host twin.

The reference rules being reproduced: event order line-then-pattern (AnalysisService.java:89-113),
events only on owned lines of a segment, penalty-before-record ranks (ScoringService.java:84-88),
context windows clipped to the document (AnalysisService.java:132-156)."""
import random

import numpy as np
import pytest
import torch

from log_parser_amd.engine import Engine, Segments
from log_parser_amd.frequency import FrequencyState
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


def _setup(n_pat, n_lines, seed, device):
    sets, trig = make_library(n_pat, seed=seed)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = Engine(lib, Config.load(overrides={"engine.device": str(device)}), device=device)
    docs = [make_log(n_lines + 37 * d, trig, seed=seed + d, hit_rate=0.08) for d in range(3)]
    data = "\n".join(docs).encode()
    size = K.padded_len(len(data))
    t = torch.zeros(size, dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(device)
    ls, ll = K.split_lines(t, len(data))
    return eng, lib, t, len(data), ls, ll


def _segments(L, rng, device):
    """3 segments with halos: [lo, hi) available, [own_lo, own_hi) owned."""
    cuts = sorted(rng.sample(range(1, L - 1), 2))
    b = [0] + cuts + [L]
    lo, hi, olo, ohi = [], [], [], []
    for i in range(3):
        lo.append(b[i])
        hi.append(b[i + 1])
        olo.append(min(b[i] + rng.randint(0, 5), b[i + 1]))
        ohi.append(max(b[i + 1] - rng.randint(0, 5), olo[-1]))
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=device)  # noqa: E731
    i64 = lambda v: torch.tensor(v, dtype=torch.int64, device=device)  # noqa: E731
    return Segments(i32(lo), i32(hi), i32(olo), i32(ohi), i64([0, 0, 0]), i64([h - l for l, h in zip(lo, hi)]))


def _reference(eng, lib, cand_hits, segs, L):
    """Plain Python version of the post-match rules over verified unique hit keys."""
    hits = sorted(set(int(k) for k in cand_hits))
    lo, hi = segs.lo.cpu().tolist(), segs.hi.cpu().tolist()
    olo, ohi = segs.own_lo.cpu().tolist(), segs.own_hi.cpu().tolist()
    seg_of = lambda x: max(i for i in range(len(lo)) if lo[i] <= x)  # noqa: E731
    prim_off = lib.prim_off
    events = []
    for k in hits:
        r, x = k >> 32, k & 0xFFFFFFFF
        s = seg_of(x)
        if not (olo[s] <= x < ohi[s]):
            continue
        for p in lib.prim_pats[prim_off[r]:prim_off[r + 1]]:
            events.append((x, int(p), s))
    events.sort()
    seen = {}
    ranks, fkeys = [], []
    cover = np.zeros(L + 1, np.int64)
    for x, p, s in events:
        fk = int(lib.freq_key[p])
        if fk >= 0:
            ranks.append(seen.get(fk, 0))
            seen[fk] = seen.get(fk, 0) + 1
        else:
            ranks.append(-1)
        fkeys.append(fk)
        b, a = int(lib.ctx_before[p]), int(lib.ctx_after[p])
        wa, wb = (x, x + 1) if b < 0 else (max(lo[s], x - b), min(hi[s], x + 1 + a))
        if wa < wb:
            cover[wa] += 1
            cover[wb] -= 1
    counts = np.zeros(max(len(lib.freq_ids), 1), np.int64)
    for fk, c in seen.items():
        counts[fk] = c
    return hits, events, ranks, fkeys, counts, np.cumsum(cover)[:L] > 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_post_pipeline_host_twin_matches_reference(seed):
    dev = torch.device("cpu")
    rng = random.Random(seed)
    eng, lib, t, n, ls, ll = _setup(60, 400, seed, dev)
    L = ls.numel()
    segs = _segments(L, rng, dev)
    cand, pre = eng.match_candidates(t, n, ls, ll)
    # duplicate some candidates and add pre-verified copies of verified hits
    verified = eng.match_hits(t, n, ls, ll)
    extra = verified[torch.randperm(verified.numel())[:verified.numel() // 3]]
    cand = torch.cat([cand, cand[: cand.numel() // 2], extra])
    evt = K.ev_tables(eng.tabs, segs, len(lib.freq_ids), len(lib.patterns))
    hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne = K.post_hits(
        cand, cand.numel() - extra.numel(), L, lib.n_regexes, t, ls, ll, eng.tabs["dfa"], evt, None)
    ref_hits, ref_ev, ref_rank, ref_fk, ref_counts, ref_cov = _reference(eng, lib, verified.tolist(), segs, L)
    assert hits.tolist() == ref_hits
    assert hit_line[:nh].tolist() == [k & 0xFFFFFFFF for k in ref_hits]
    for r in range(lib.n_regexes + 1):
        assert int(hit_off[r]) == sum(1 for k in ref_hits if (k >> 32) < r)
    assert ne == len(ref_ev)
    ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, counts, feat, cov = K.post_events(
        hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll, eng.tabs["dfa"], len(lib.freq_ids), None, features=False)
    assert list(zip(ev_line.tolist(), ev_pat.tolist(), ev_seg.tolist())) == ref_ev
    assert ev_rank.tolist() == ref_rank and ev_fkey.tolist() == ref_fk
    assert counts.tolist() == ref_counts.tolist()
    assert ((cov[:L] > 0).numpy() == ref_cov).all()
    # features: only covered lines are evaluated, the rest stay 0
    *_, feat2, _ = K.post_events(hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll, eng.tabs["dfa"],
                                 len(lib.freq_ids), None, features=True)
    from log_parser_amd import golden
    raw = bytes(t[:n].tolist())
    full = []
    for a, b in zip(ls.tolist(), ll.tolist()):      # ContextAnalysisService.java:62-83 per line
        line = raw[a:a + b].decode("utf-8", errors="replace")
        f = 1 if golden._find(golden.ERROR_RE, line) else (2 if golden._find(golden.WARN_RE, line) else 0)
        f |= (4 if golden._find(golden.STACK_RE, line) else 0) | (8 if golden._find(golden.EXC_RE, line) else 0)
        full.append(f)
    full = torch.tensor(full, dtype=torch.uint8)
    assert torch.equal(feat2[:L], torch.where(torch.from_numpy(ref_cov), full, torch.zeros_like(full)))


def test_post_pipeline_empty_inputs():
    dev = torch.device("cpu")
    eng, lib, t, n, ls, ll = _setup(10, 50, 7, dev)
    L = ls.numel()
    segs = Segments.single(L, dev)
    evt = K.ev_tables(eng.tabs, segs, len(lib.freq_ids), len(lib.patterns))
    empty = torch.empty(0, dtype=torch.int64)
    hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne = K.post_hits(empty, 0, L, lib.n_regexes, t, ls, ll,
                                                                  eng.tabs["dfa"], evt, None)
    assert nh == 0 and ne == 0 and hit_off.tolist() == [0] * (lib.n_regexes + 1)
    out = K.post_events(hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll, eng.tabs["dfa"], len(lib.freq_ids), None)
    assert out[0].numel() == 0 and int(out[6][:L].sum()) == 0


def test_frequency_state_vectorised_semantics():
    t = [0.0]
    st = FrequencyState(1, clock=lambda: t[0])
    ids = ["a", "b", "c"]
    st.record_counts(ids, np.array([3, 0, 1]))
    t[0] = 1800.0
    st.record_counts(ids, np.array([2, 5, 0]))
    assert st.carry(ids).tolist() == [5, 5, 1]
    assert st.get_pattern_frequency("b") == {"patternId": "b", "currentCount": 5, "hourlyRate": 5.0}
    snap = st.capture()
    t[0] = 3600.5                                    # first batch leaves the window
    assert st.carry(ids).tolist() == [2, 5, 0]
    st.reset("b")
    assert st.carry(ids).tolist() == [2, 0, 0] and st.get_pattern_frequency("b")["currentCount"] == 0
    t[0] = 5400.5                                    # second batch leaves: no negative counts after reset
    assert st.carry(ids).tolist() == [0, 0, 0]
    assert st.statistics() == {"a": 0, "b": 0, "c": 0}
    st.rollback(snap)
    t[0] = 1800.0
    assert st.carry(ids).tolist() == [5, 5, 1]
    st.reset_all()
    assert st.get_pattern_frequency("a") is None and st.carry(["a", "zz"]).tolist() == [0, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_post_pipeline_gpu_equals_host_twin(gpu_device, seed):
    rng = random.Random(seed)
    eng_d, lib, td, n, ls_d, ll_d = _setup(200, 3000, seed, gpu_device)
    eng_c = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    tc, ls_c, ll_c = td.cpu(), ls_d.cpu(), ll_d.cpu()
    L = ls_c.numel()
    segs_c = _segments(L, rng, torch.device("cpu"))
    segs_d = Segments(*(getattr(segs_c, f).to(gpu_device) for f in ("lo", "hi", "own_lo", "own_hi", "g0", "n")))
    pd = eng_d.prepare(td, n, ls_d, ll_d, segs_d)
    pc = eng_c.prepare(tc, n, ls_c, ll_c, segs_c)
    assert torch.equal(pd.hits.cpu(), pc.hits)
    assert torch.equal(pd.hit_off.cpu(), pc.hit_off)
    for f in ("ev_line", "ev_pat", "ev_seg", "ev_rank", "ev_fkey", "freq_counts"):
        assert torch.equal(getattr(pd, f).cpu(), getattr(pc, f)), f
    assert torch.equal(pd.feat[:L].cpu(), pc.feat[:L])
    carry = torch.arange(max(len(lib.freq_ids), 1), dtype=torch.int64) * 3
    rd = eng_d.finish(pd, segs_d, carry.to(gpu_device))
    rc = eng_c.finish(pc, segs_c, carry)
    assert torch.equal(rd.score.cpu(), rc.score)     # bit-identical fp64 (no FMA contraction either side)


@pytest.mark.parametrize("seed", [0, 1])
def test_pack_split_docs_sliced_large_documents(seed):
    """Large documents are copied/split in 256 KiB slices on several threads: slice boundaries
    inside '\\r\\n', runs of empty lines and trailing empties must still give Java's split."""
    from log_parser_amd import golden
    from log_parser_amd.native import N
    rng = random.Random(seed)
    docs = []
    for _ in range(4):
        parts = []
        size = 0
        target = rng.randint(2_000_000, 4_000_000)   # > 4 MB total per thread: several threads
        while size < target:
            x = rng.choice(["a", "line with words", "\r", "é", ""]) * rng.randint(0, 30) + \
                rng.choice(["\n", "\r\n", "\n\n\n", "\r\n\r\n"])
            parts.append(x)
            size += len(x)
        docs.append("".join(parts) + rng.choice(["", "\n\n\n", "\r\n", "tail", "\n\r"]))
    docs.append("\n" * 600_000)                      # only empty lines: zero kept lines
    docs.append("x" * 700_000)                        # no newline at all: one line
    total = sum(len(d.encode()) for d in docs)
    buf = np.zeros(total + 64, np.uint8)
    for nthreads in (1, 4, 16):
        ls, ll, dl, off = N.pack_split_docs(docs, buf.ctypes.data, buf.size, nthreads)
        raw = buf.tobytes()
        for d, doc in enumerate(docs):
            got = [raw[a:a + b].decode() for a, b in zip(ls[dl[d]:dl[d + 1]], ll[dl[d]:dl[d + 1]])]
            assert got == golden.split_lines(doc), (nthreads, d)


def test_native_batch_results_match_golden_and_uuid4():
    """emit_batch_results (csrc/io/json_emit.cpp) writes the whole AnalysisResult natively:
    version-4 UUIDs unique per response, metadata, and the summary of every document equal to the
    sequential golden model (severity histogram, highest severity incl. unknown severities)."""
    import json
    import re
    from log_parser_amd import golden
    sets, trig = make_library(30, seed=17)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    docs = [make_log(150 + 40 * i, trig, seed=170 + i, hit_rate=0.1 * (i % 3)) for i in range(7)] + ["", "\n\n"]
    outs = [json.loads(o) for o in eng.analyze_batch_json(docs)]
    tracker = golden.FrequencyTracker(ScoringParams())
    ids = set()
    for d, o in zip(docs, outs):
        g = golden.analyze(d, sets, ScoringParams(), tracker)
        assert re.fullmatch(r"[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}", o["analysisId"])
        ids.add(o["analysisId"])
        assert o["summary"] == g["summary"]
        assert o["metadata"]["totalLines"] == g["metadata"]["totalLines"]
        assert o["metadata"]["patternsUsed"] == g["metadata"]["patternsUsed"]
        assert [e["score"] for e in o["events"]] == pytest.approx([e["score"] for e in g["events"]], rel=1e-12)
    assert len(ids) == len(docs)
