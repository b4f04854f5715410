"""Prefilter tables (models/compiled.py _build_prefilter): with stride-S sampling (S = 2 or 4) every
literal indexes S adjacent 4-byte windows, so every occurrence of a literal has an indexed window that
starts at a text position divisible by S -- the positions k_prefilter<16, S> tests. Checked here on the
tables themselves (the device kernel is covered by the GPU tests against the golden model)."""
import random

import numpy as np
import pytest

from log_parser_amd.models import compiled as C
from log_parser_amd.utils.config import ScoringParams
from log_parser_amd.utils.synth import make_library


def _entries(pf):
    H = pf["ht_mask"] + 1
    out = {}
    for h in range(H):
        k = int(pf["ht_key"][h])
        if k == 2 ** 64 - 1:
            continue
        key, g = k & 0xFFFFFFFF, k >> 32
        for j in range(int(pf["ht_cnt"][h])):
            e = int(pf["gram_lits"][int(pf["ht_val"][h]) + j])
            out.setdefault(e & ((1 << C.LIT_OFF_SHIFT) - 1), []).append((key, g, e >> C.LIT_OFF_SHIFT))
    return out


def _lib_with_max_stride(smax, n=200, seed=5, teddy=True):
    old = C.PF_STRIDE_MAX, C.PF_TEDDY
    try:
        C.PF_STRIDE_MAX, C.PF_TEDDY = smax, teddy
        sets, _ = make_library(n, seed=seed)
        return C.CompiledLibrary(sets, ScoringParams())
    finally:
        C.PF_STRIDE_MAX, C.PF_TEDDY = old


@pytest.mark.parametrize("S", [2, 4])
def test_strided_tables_index_adjacent_windows_and_bloom_holds_them(S):
    lib = _lib_with_max_stride(S)
    pf = lib.pf
    assert pf["stride"] == S                          # synthetic literals have >= 9 bytes
    ents = _entries(pf)
    assert set(ents) == set(range(len(lib.literals)))
    for i, lit in enumerate(lib.literals):
        offs = sorted(o for _, _, o in ents[i])
        assert offs == list(range(offs[0], offs[0] + S)) and offs[-1] + 4 <= len(lit)
        for key, g, o in ents[i]:
            assert g == 4 and key == int.from_bytes(lit[o:o + 4], "little")
            w = C.bloom_word(key, g, pf["bits"])
            m = C.bloom_bits2(key, g)
            assert int(pf["bloom"][w]) & m == m


@pytest.mark.parametrize("S", [2, 4])
def test_every_occurrence_hits_a_tested_position(S):
    lib = _lib_with_max_stride(S, n=60, seed=9)
    assert lib.pf["stride"] == S
    ents = _entries(lib.pf)
    rng = random.Random(3)
    for i, lit in enumerate(lib.literals[:200]):
        for shift in range(S):
            q = rng.randrange(0, 40) * S + shift           # occurrence at every residue mod S
            starts = [q + o for _, _, o in ents[i]]
            assert sum(p % S == 0 for p in starts) == 1    # exactly one indexed window is tested


def _one(regex, teddy=True):
    import yaml
    from log_parser_amd.models.schema import PatternSet
    doc = yaml.safe_load(f"""
metadata: {{library_id: s}}
patterns:
  - id: p1
    name: one literal
    severity: HIGH
    primary_pattern: {{regex: "{regex}", confidence: 0.9}}
""")
    old = C.PF_TEDDY
    try:
        C.PF_TEDDY = teddy
        return C.CompiledLibrary([PatternSet.model_validate(doc)], ScoringParams())
    finally:
        C.PF_TEDDY = old


def test_short_literals_go_to_the_teddy_tier():
    """3..6-byte literals use the byte-position tier and leave the bloom tier at stride 4."""
    lib = _one("OOMKil")
    assert lib.pf["teddy_lits"] == 1 and lib.pf["gmask"] == 0
    lib = _one("(OOM|SIGSEGVKILL)")
    assert lib.pf["teddy_lits"] == 1 and lib.pf["stride"] == 4      # "sigsegvkill" on the bloom tier
    assert _one("ab").summary()["scan_all"] == 1                     # < 3 bytes: scan every line


@pytest.mark.parametrize("seed", [1, 2])
def test_teddy_masks_hold_every_short_window(seed):
    from log_parser_amd.utils.synth import realistic_library
    sets, _ = realistic_library(300, seed=seed)
    lib = C.CompiledLibrary(sets, ScoringParams())
    pf = lib.pf
    assert pf["teddy_lits"] > 5
    tab, off, ent = pf["teddy"], pf["tb_off"], pf["tb_lits"]
    seen = set()
    for b in range(C.TEDDY_BUCKETS):
        for e in ent[off[b]:off[b + 1]]:
            i, o = int(e) & ((1 << C.LIT_OFF_SHIFT) - 1), int(e) >> C.LIT_OFF_SHIFT
            lit = lib.literals[i]
            assert C.TEDDY_MIN <= len(lit) <= C.TEDDY_MAX and o + 3 <= len(lit)
            for j in range(3):
                assert int(tab[lit[o + j], j]) >> b & 1
            seen.add(i)
    assert len(seen) == pf["teddy_lits"]


def test_every_short_occurrence_is_a_candidate_cpu():
    """Host prefilter twin: each planted short literal (any case, any alignment) yields its
    (regex, line) candidate; the bloom tier yields one candidate per long-literal occurrence."""
    import torch
    from log_parser_amd.ops import kernels as K
    lib = _one("(?i)qx7|VERYLONGLITERAL")
    lines = [b"noise", b"a QX7 b", b"xqx7", b"verylongliteral here", b"q x7"]
    data = b"\n".join(lines)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    cand = K.prefilter(t, len(data), lib.device_tables(torch.device("cpu"))["pf"], ls, 64)
    got = sorted(set(int(c) & 0xFFFFFFFF for c in cand.tolist()))
    assert got == [1, 2, 3]
    assert cand.numel() == 3                          # no duplicate per indexed window


def test_stride_follows_the_shortest_literal():
    def lib_for(regex):
        return _one(regex, teddy=False)
    assert lib_for("OOMKill").pf["stride"] == 4       # 7 bytes: four 4-byte windows
    assert lib_for("OOMKil").pf["stride"] == 2        # 6 bytes: only three windows
    assert lib_for("OOMK").pf["stride"] == 1


def test_short_literals_fall_back_to_stride1():
    old = C.PF_STRIDE_MAX, C.PF_TEDDY
    try:
        C.PF_STRIDE_MAX, C.PF_TEDDY = 1, False
        sets, _ = make_library(30, seed=5)
        assert C.CompiledLibrary(sets, ScoringParams()).pf["stride"] == 1
    finally:
        C.PF_STRIDE_MAX, C.PF_TEDDY = old
    lib = _one("OOM", teddy=False)
    assert lib.pf["stride"] == 1                      # a 3-byte literal has no two 4-byte windows
    assert np.all(np.array([len(l) for l in lib.literals]) >= 1)


def _parity_run(dev, lib, data, torch):
    from log_parser_amd.engine import Engine, Segments
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.config import Config
    eng = Engine(lib, Config.load(overrides={"engine.device": str(dev)}), device=dev)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(dev)
    ls, ll = K.split_lines(t, len(data))
    res = eng.run(t, len(data), ls, ll, Segments.single(ls.numel(), dev), eng.freq_carry())
    return res.ev_line.cpu().numpy(), res.ev_pat.cpu().numpy(), res.score.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("smax,teddy", [(1, False), (2, False), (4, False), (4, True)])
def test_every_prefilter_variant_gpu_equals_cpu_and_golden(gpu_device, smax, teddy):
    """Pins each k_prefilter<GM, S, *, TD> variant on the device: the library's sampling stride
    (1, 2 or 4, from PF_STRIDE_MAX) and the Teddy tier on/off, against the host twin and the
    golden model (AnalysisService.java:89-95 runs every primary on every line)."""
    import torch
    from log_parser_amd import golden
    from log_parser_amd.utils.synth import make_log, realistic_library
    old = C.PF_STRIDE_MAX, C.PF_TEDDY
    try:
        C.PF_STRIDE_MAX, C.PF_TEDDY = smax, teddy
        sets, trig = realistic_library(150, seed=23) if teddy else make_library(150, seed=23)
        lib = C.CompiledLibrary(sets, ScoringParams())
    finally:
        C.PF_STRIDE_MAX, C.PF_TEDDY = old
    assert lib.pf["stride"] == smax and bool(lib.pf["teddy_lits"]) == teddy
    logs = make_log(4000, trig, seed=24, hit_rate=0.05, crlf_rate=0.1)
    data = logs.encode()
    g = _parity_run(gpu_device, lib, data, torch)
    c = _parity_run(torch.device("cpu"), lib, data, torch)
    for a, b in zip(g, c):
        np.testing.assert_array_equal(a, b)
    ref = golden.analyze(logs, sets, ScoringParams(), golden.FrequencyTracker(ScoringParams()))
    assert [(e["lineNumber"] - 1, e["matchedPattern"]["id"]) for e in ref["events"]] == \
        [(int(x), lib.patterns[int(p)].id) for x, p in zip(g[0], g[1])]
    np.testing.assert_allclose(g[2], [e["score"] for e in ref["events"]], rtol=1e-12)


@pytest.mark.parametrize("S", [1, 2, 4])
def test_host_prefilter_simd_equals_exact_literal_search(S):
    """The CPU backend's bloom tier (AVX-512, 16 positions per step, prefilter_cpu.cpp) finds every
    literal occurrence: its candidates == an exact search for every library literal on every line,
    with occurrences at every residue mod 64 (step edges), mixed case, the text end and no-hit text."""
    import torch
    from log_parser_amd.ops import kernels as K
    lib = _lib_with_max_stride(S, n=40, seed=11, teddy=False)
    assert lib.pf["stride"] == S and lib.pf["gmask"] == 16
    tabs = lib.device_tables(torch.device("cpu"))
    rng = random.Random(S)
    lines = []
    for i in range(3000):
        pad = "x" * rng.randrange(0, 130)
        if rng.random() < 0.1:
            lit = rng.choice(lib.literals).decode("latin-1")
            lit = lit.upper() if rng.random() < 0.3 else lit
            lines.append(pad + lit + "y" * rng.randrange(0, 5))
        else:
            lines.append(pad + "noise line %d" % i)
    lines.append("tail " + lib.literals[0].decode("latin-1"))        # literal touching the text end
    data = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    got = set(K.prefilter(t, len(data), tabs["pf"], ls, 1 << 16).tolist())
    # exact: (regex << 32 | line) for every literal occurring (case-insensitively) in a line
    lit_regs = {}
    for i, lit in enumerate(lib.literals):
        a, b = int(lib.pf["lit_reg_off"][i]), int(lib.pf["lit_reg_off"][i + 1])
        lit_regs[lit.lower()] = [int(r) for r in lib.pf["lit_reg"][a:b]]
    want = set()
    for x, line in enumerate(data.split(b"\n")):
        low = line.lower()
        for lit, regs in lit_regs.items():
            if lit in low:
                want.update((r << 32) | x for r in regs)
    assert got == want and len(want) > 100


def test_host_prefilter_simd_teddy_equals_exact_literal_search():
    """Both tiers on the CPU backend (AVX-512 bloom tier for the long literals, three-gather Teddy tier
    for the 3-6-byte ones): candidates == an exact literal search on every line."""
    import torch
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.synth import realistic_library
    sets, trig = realistic_library(120, seed=5)
    lib = C.CompiledLibrary(sets, ScoringParams())
    assert lib.pf["teddy_lits"] > 0 and lib.pf["gmask"] == 16
    tabs = lib.device_tables(torch.device("cpu"))
    rng = random.Random(21)
    lines = []
    for i in range(4000):
        pad = "q" * rng.randrange(0, 90)
        if rng.random() < 0.15:
            lit = rng.choice(lib.literals).decode("latin-1")
            lit = lit.upper() if rng.random() < 0.3 else lit
            lines.append(pad + lit + "z" * rng.randrange(0, 4))
        else:
            lines.append(pad + "plain text %d" % i)
    lines.append(lib.literals[-1].decode("latin-1"))
    data = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    got = set(K.prefilter(t, len(data), tabs["pf"], ls, 1 << 18).tolist())
    lit_regs = {}
    for i, lit in enumerate(lib.literals):
        a, b = int(lib.pf["lit_reg_off"][i]), int(lib.pf["lit_reg_off"][i + 1])
        lit_regs.setdefault(lit.lower(), []).extend(int(r) for r in lib.pf["lit_reg"][a:b])
    want = set()
    for x, line in enumerate(data.split(b"\n")):
        low = line.lower()
        for lit, regs in lit_regs.items():
            if lit in low:
                want.update((r << 32) | x for r in regs)
    assert got == want and len(want) > 100


def test_fingerprints_never_reject_an_occurrence():
    """k_pf_verify skips a bucket literal when the 8 text bytes around the window (4 before, 4
    after, lower-cased) disagree with its fingerprint under its mask: every true occurrence of
    every literal must pass, for both tiers (bloom windows g = 4, Teddy windows g = 3)."""
    import random
    import numpy as np
    from log_parser_amd.models.compiled import CompiledLibrary, LIT_OFF_SHIFT
    from log_parser_amd.utils.config import ScoringParams
    from log_parser_amd.utils.synth import realistic_library
    sets, _ = realistic_library(300, seed=3)
    lib = CompiledLibrary(sets, ScoringParams())
    pf = lib.pf
    rng = random.Random(1)

    def t8_at(text: bytes, p: int, g: int) -> int:
        low = bytes(text).lower()
        before = sum((low[p - 4 + k] if p - 4 + k >= 0 else 0) << (8 * k) for k in range(4))
        after = sum((low[p + g + k] if p + g + k < len(low) else 0) << (8 * k) for k in range(4))
        return before | (after << 32)

    def check(ents, fps, gs):
        n = 0
        for j, e in enumerate(ents):
            lit = lib.literals[int(e) & ((1 << LIT_OFF_SHIFT) - 1)]
            off = int(e) >> LIT_OFF_SHIFT
            assert lit[off:off + gs[j]].lower() == lit[off:off + gs[j]]
            pre = bytes(rng.choice(b"abc xyZ09:") for _ in range(rng.randint(0, 9)))
            text = pre + lit.upper() if rng.random() < 0.5 else pre + lit
            text += bytes(rng.choice(b"qrs_ 7") for _ in range(rng.randint(0, 9)))
            t8 = t8_at(text, len(pre) + off, int(gs[j]))
            fp, mask = int(fps[2 * j]), int(fps[2 * j + 1])
            assert (t8 ^ fp) & mask == 0, (lit, off)
            n += mask != 0
        return n
    assert check(pf["gram_lits"], pf["gram_fp"], pf["gram_g"]) > 100
    ntb = int(pf["tb_off"][-1])
    check(pf["tb_lits"][:ntb], pf["tb_fp"], [3] * ntb)
