"""Bit-parallel Glushkov programs over code points (jregex.cpp bpg_program, csrc/kernels/bpg.h) for
regexes whose DFA blows up -- bounded gaps ``X.{0,1000}Y``, repeated groups, boundary-gated edges --
or that need code-point contexts (MULTILINE ``^ $``, Unicode ``\b``). The reference runs
``Pattern.compile(rx).matcher(line).find()`` for every regex role (AnalysisService.java:62-65,93-95;
secondaries ScoringService.java:315-347), so these must give exactly Java's boolean find():
checked against the javacompat oracle (pure Python twin, native host twin, gfx950 kernel) and end
to end against the golden model."""
import random

import numpy as np
import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine
from log_parser_amd.models.bpg import program_info, run_program
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.native import N
from log_parser_amd.ops import kernels as K
from log_parser_amd.regex.javacompat import compile_java
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log

GAP_PATS = [
    r"Connection refused.{0,120}port \d+", r"pod .{1,60} in namespace .{1,60} failed",
    r"error.{0,100}timeout.{0,100}retry", r"(\w+\.){2,}\w+Exception.{0,200}Caused by",
    r"(?i)\bfoo\b.{0,40}bar", r"x.{0,3}y", r"^\s*at .{0,50}\(", r"(?i)(?:fail|error|fatal).{0,30}(?:disk|volume|mount)\b",
    r"\b\d{1,3}(?:\.\d{1,3}){3}\b.{0,80}(?:refused|reset|timed out)", r"(a|bc)+d.{0,20}e", r"a.{2,5}b$",
    r"(?i)é.{0,9}z\B", r"(?:ab|cd){2,4}.{0,30}x+y?z",
    # wide gaps (> 512 positions at byte level), MULTILINE anchors, Unicode classes / \b
    r"Connection refused.{0,600}port \d+", r"error.{0,300}timeout.{0,300}retry", r"X.{0,1000}Y",
    r"(?m)^ERROR$", r"(?m)fail$.{0,5}", r"(?U)\bfoo\w*\b.{0,20}bar", r"\p{L}+Exception.{0,50}at",
    r"[^é]x.{0,40}y", r"(?iu)ÉCOLE.{0,30}\p{Lu}",
]
POS = ["Connection refused by 10.0.0.1 on port 80", "pod a in namespace b c failed", "error: x timeout y retry",
       "at com.acme.FooException: bad Caused by", "FOO, then bar", "x12y", "  at x(", "Fatal: no disk",
       "10.0.0.1 said hi refused", "abcbcd123e", "aééb", "ÉabcZz", "abcd...xxz",
       "Connection refused " + "x" * 580 + "port 8", "error " + "é" * 280 + "timeout" + "y" * 250 + "retry",
       "X" + "z" * 990 + "Y", "boom\rERROR", "ERROR\u2028x", "it fail\u0085", "fooé bar", "féoo xbar",
       "ÉcoleException at", "zx oy", "école 1 Ä"]
ALPHA = "abcdefxyz .:()é\tÉ" + "Connection refused port 123 pod in namespace failed error timeout retry " \
        "java.lang.FooException Caused by foo bar FOO at 10.0.0.1 disk volume\r" \
        "ERROR fail X Y \u0085\u2028\u2029 école ÉCOLE Ä 日本 x y"


def _lines(rng, n):
    toks = ALPHA.split(" ")
    out = list(POS)
    for _ in range(n):
        if rng.random() < 0.5:
            out.append(" ".join(rng.choice(toks) for _ in range(rng.randint(0, 25))))
        else:
            out.append("".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 90))))
    return out


def test_decomposition_is_exact_and_compact():
    """jregex builds every shape into an exact program (bpg_program checks the decomposition) with
    few exception rows; the wide bounded gaps need none."""
    for p in GAP_PATS:
        d = N.compile_regex(p, 64, 4096)
        assert d["kind"] in (0, 1), (p, d["error"])
        if d["kind"] == 1:
            assert d["bpg"], (p, d["error"])
            assert program_info(d["bpg"])["exceptions"] <= 4, (p, program_info(d["bpg"]))
    for p in GAP_PATS[:3] + GAP_PATS[13:16]:
        d = N.compile_regex(p, 2048, 4096)
        assert d["kind"] == 1 and program_info(d["bpg"])["exceptions"] == 0, p
    # a bounded repeat of one class is ONE counted position; repeated groups stay expanded
    info = program_info(N.compile_regex(r"X.{0,1000}Y")["bpg"])
    assert info["words"] == 1 and info["counters"] == 1
    info = program_info(N.compile_regex(r"X(?:a.){0,500}Y")["bpg"])
    assert info["words"] == 16 and info["counters"] == 0


@pytest.mark.parametrize("seed", [0, 1])
def test_python_twin_matches_java_oracle(seed):
    rng = random.Random(seed)
    lines = _lines(rng, 400)
    for p in GAP_PATS:
        d = N.compile_regex(p, 64, 4096)
        if d["kind"] != 1:
            continue
        rx = compile_java(p)
        for s in lines:
            want = rx.search(s) is not None
            assert run_program(d["bpg"], s.encode()) == want, (p, s)
            assert N.bpg_find(d["bpg"], s.encode()) == want, (p, s)


def _lib(pats):
    from log_parser_amd.models.schema import PatternSet
    ps = PatternSet.model_validate({"metadata": {"library_id": "gap"}, "patterns": [
        {"id": f"g{i}", "name": p, "severity": "HIGH", "primary_pattern": {"regex": p, "confidence": 0.5}}
        for i, p in enumerate(pats)]})
    return CompiledLibrary([ps], ScoringParams(), max_dfa_states=64)


def _scan(lib, lines, dev):
    blob = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(blob)), dtype=torch.uint8)
    t[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    starts, lens, pos = [], [], 0
    for s in lines:
        starts.append(pos)
        lens.append(len(s.encode()))
        pos += lens[-1] + 1
    ls = torch.tensor(starts, dtype=torch.int64, device=dev)
    ll = torch.tensor(lens, dtype=torch.int32, device=dev)
    tabs = lib.device_tables(dev)
    regs = torch.tensor(lib.bpg_regs, dtype=torch.int32, device=dev)
    return set(K.scan(t.to(dev), ls, ll, regs, tabs["dfa"], 1 << 16).cpu().tolist())


def test_native_host_twin_matches_oracle():
    lib = _lib(GAP_PATS)
    assert len(lib.bpg_regs) >= len(GAP_PATS) - 2   # max_dfa_states=64: nearly all are BPG programs
    lines = _lines(random.Random(5), 600)
    got = _scan(lib, lines, torch.device("cpu"))
    want = {(r << 32) | j for r in lib.bpg_regs for j, s in enumerate(lines)
            if compile_java(lib.regexes[r].pattern).search(s) is not None}
    assert got == want and len(want) > 50


def _gap_library(seed):
    sets, trig = make_library(48, seed=seed, gap_rate=0.5)
    return sets, trig


@pytest.mark.parametrize("seed", [11, 12])
def test_engine_with_bounded_gap_regexes_matches_golden(seed):
    """Bounded-gap primaries (literal-narrowed to prefilter candidates) and bounded-gap
    secondaries give the golden model's events and scores (rtol 1e-12); nothing runs on the host
    backtracker and the native request runner stays eligible."""
    p = ScoringParams()
    sets, trig = _gap_library(seed)
    lib = CompiledLibrary(sets, p)
    s = lib.summary()
    assert s["nfa_bpg"] >= 10 and s["host_fallback"] == 0 and s["nfa_mfma"] == 0
    logs = make_log(4000, trig, seed=seed + 1, hit_rate=0.08, crlf_rate=0.05)
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    r = eng.analyze(logs)
    g = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in r["events"]] == \
        [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
    gap_ids = {pt.id for ps in sets for pt in ps.patterns if "{" in pt.primary_pattern.regex}
    assert sum(e["matchedPattern"]["id"] in gap_ids for e in r["events"]) > 20
    np.testing.assert_allclose([e["score"] for e in r["events"]], [e["score"] for e in g["events"]], rtol=1e-12)


@pytest.mark.gpu
def test_bpg_kernel_matches_host(gpu_device):
    lib = _lib(GAP_PATS)
    lines = _lines(random.Random(6), 5000)
    assert _scan(lib, lines, gpu_device) == _scan(lib, lines, torch.device("cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11])
def test_engine_bounded_gap_gpu_matches_golden(gpu_device, seed):
    p = ScoringParams()
    sets, trig = _gap_library(seed)
    lib = CompiledLibrary(sets, p)
    logs = make_log(4000, trig, seed=seed + 1, hit_rate=0.08)
    eng = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device)}), device=gpu_device)
    r = eng.analyze(logs)
    assert eng._runner not in (None, False)            # the native request runner served it
    g = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in r["events"]] == \
        [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
    np.testing.assert_allclose([e["score"] for e in r["events"]], [e["score"] for e in g["events"]], rtol=1e-12)


# libraries whose widest program sets the wave-cooperative group size (bpg.hip k_bpg_coop<G>):
# 1 word -> G = 2 lanes, 2 words -> 4, up to 4 words -> 8, 6 / 8 words -> 16 (exceptions and boundary-gated
# programs included)
COOP_LIBS = [
    ([r"ab.{0,10}cd", r"x.{0,3}y", r"(a|bc)+d.{0,20}e", r"(?i)é.{0,3}z\B"], 8),
    (GAP_PATS[4:6], 64),
    (GAP_PATS[4:], 64),
    (GAP_PATS[:13] + [r"a(?:é.){0,75}b", r"(?i)error(?: .){0,110}\bdisk"], 64),
    (GAP_PATS + [r"a(?:é.){0,400}b"], 64),            # up to 16 words -> G = 32 (+ counted gaps)
    ([r"a(?:é.){0,700}b", r"(?m)^x$", r"a.{0,1500}b"], 64),   # 24 words -> G = 64
]


def _text_dev(lines, dev):
    blob = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(blob)), dtype=torch.uint8)
    t[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    starts, lens, pos = [], [], 0
    for s in lines:
        starts.append(pos)
        lens.append(len(s.encode()))
        pos += lens[-1] + 1
    return (t.to(dev), torch.tensor(starts, dtype=torch.int64, device=dev),
            torch.tensor(lens, dtype=torch.int32, device=dev))


@pytest.mark.gpu
@pytest.mark.parametrize("li", range(len(COOP_LIBS)))
def test_bpg_candidate_walks_match_host(gpu_device, li):
    """The candidate walks (request path: in-place verify; bulk path: first-of-run flags over sorted
    keys with duplicates and pre-verified copies) give the host twin's find() for every width."""
    pats, max_states = COOP_LIBS[li]
    from log_parser_amd.models.schema import PatternSet
    ps = PatternSet.model_validate({"metadata": {"library_id": "gap"}, "patterns": [
        {"id": f"g{i}", "name": p, "severity": "HIGH", "primary_pattern": {"regex": p, "confidence": 0.5}}
        for i, p in enumerate(pats)]})
    lib = CompiledLibrary([ps], ScoringParams(), max_dfa_states=max_states)
    assert lib.bpg_regs
    rng = random.Random(40 + li)
    lines = _lines(rng, 3000) + ["a" + "é" * k + "b" for k in range(0, 160, 7)] + \
        ["ERROR " + "x" * k + " disk" for k in range(0, 260, 13)]
    text, ls, ll = _text_dev(lines, gpu_device)
    dfa = lib.device_tables(gpu_device)["dfa"]
    progs = {r: lib.bpg_program(r).tobytes() for r in lib.bpg_regs}      # the C++ host twin (bpg.h)
    want = {(r, j) for r in lib.bpg_regs for j, s in enumerate(lines) if N.bpg_find(progs[r], s.encode())}
    assert len(want) > 50
    # request path: every (regex, line) pair plus rejected slots (-1) and non-BPG regexes, shuffled
    pairs = [(r, j) for r in lib.bpg_regs for j in range(len(lines))]
    others = [r for r in range(len(lib.regexes)) if r not in set(lib.bpg_regs)]
    pairs += [(others[k % len(others)], k) for k in range(0, len(lines), 5)] if others else []
    rng.shuffle(pairs)
    cand = [(r << 32) | j for r, j in pairs] + [-1] * 77
    ct = torch.tensor(cand, dtype=torch.int64, device=gpu_device)
    N.bpg_cand_dev(ct.data_ptr(), ct.numel(), text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa,
                   torch.cuda.current_stream().cuda_stream)
    got = ct.cpu().tolist()
    bpg = set(lib.bpg_regs)
    for before, after in zip(cand, got):
        if before < 0 or (before >> 32) not in bpg:
            assert after == before
        else:
            assert (after >= 0) == ((before >> 32, before & 0xFFFFFFFF) in want), (before >> 32, before & 0xFFFFFFFF)
    # bulk path: sorted packed keys, some duplicated, some pre-verified (flag bit 1)
    lbits = N.bits_for(len(lines))
    keys = []
    for r, j in pairs:
        k = ((r << lbits) | j) << 1
        keys.append(k)
        if rng.random() < 0.1:
            keys.append(k)
        if rng.random() < 0.05:
            keys.append(k | 1)
    keys.sort()
    kt = torch.tensor(keys, dtype=torch.int64, device=gpu_device)
    for listed in (False, True):    # wide programs walked in place / from the listed keys (bulk path)
        flag = torch.full((len(keys),), 7, dtype=torch.uint8, device=gpu_device)
        wcnt = torch.zeros(1, dtype=torch.int32, device=gpu_device)
        wlist = torch.zeros(len(keys), dtype=torch.int32, device=gpu_device)
        N.bpg_dedupe_dev(kt.data_ptr(), kt.numel(), lbits, text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa,
                         flag.data_ptr(), torch.cuda.current_stream().cuda_stream,
                         wcnt.data_ptr() if listed else 0, wlist.data_ptr() if listed else 0)
        fl = flag.cpu().tolist()
        pre = {}
        for x in keys:                       # run (same regex + line) -> holds a pre-verified copy
            pre[x >> 1] = pre.get(x >> 1, False) or bool(x & 1)
        for i, k in enumerate(keys):
            kk = k >> 1
            r, j = kk >> lbits, kk & ((1 << lbits) - 1)
            first = i == 0 or keys[i - 1] >> 1 != kk
            if first and r in bpg and not pre[kk]:
                assert fl[i] == (1 if (r, j) in want else 0), (r, j, listed)
            else:
                assert fl[i] == 7


# ---- counted positions: bounded repeats of one class at any bound (no 2,048-position cliff) ----
# (a leading / trailing repeat is trimmed to its minimum by find()-equivalence -- x{2,5000} is x{2},
# a DFA -- so these repeats sit behind an anchor alternative that keeps them counted)
CTR_PATS = [r"(?:^|=)x{2,5000}(?:$|=)", r"(?:^|=)[^\n]{0,2500}FATAL", r"(?i)(err|warn).{0,2100}x", r"X.{0,3000}Y", r"X.{0,20000}Y",
            r"a.{3,40}b", r"^.{0,20}é{5,50}", r"(?i)error.{0,30}tok.{0,30}retry", r"X.{0,17}Y", r"\bX.{0,16}\bY",
            r"(?:q.{0,40})+Z", r"X[^\r]{0,50}(?m)$", r"X.{0,5000}Y.{0,2100}Z"]


def _ctr_lines(rng, gap):
    """Lines around the bound: k = gap-2 .. gap+2 characters between the anchors (ASCII and
    2-byte code points), a younger re-entry past an expired older one, a line terminator inside
    the gap, and random lines up to 2 x gap long."""
    out = []
    for k in range(gap - 2, gap + 3):
        out += ["X" + "z" * k + "Y", "X" + "é" * k + "Y", "X" + "z" * (k + 5) + "X" + "z" * 10 + "Y",
                "X" + "z" * (k // 2) + "\r" + "z" * (k // 2) + "Y", "a" + "q" * k + "b", "x" * min(k, 6000),
                "err" + "." * k + "x", "é" * k + "FATAL", "X" + "z" * k + "Y" + "z" * 2000 + "Z"]
    toks = ["X", "Y", "z", "é", "\r", " ", "FATAL", "err", "WARN", "x", "xx", "a", "b", "q", "1", "22", "error", "tok",
            "retry", "Z", "日"]
    for _ in range(12):
        n = rng.randint(0, 2 * gap)
        out.append("".join(rng.choice(toks) if rng.random() < 0.05 else "z" for _ in range(n)))
    return out


@pytest.mark.parametrize("gap", [2100, 5000, 20000])
def test_counted_repeats_match_java_oracle(gap):
    """Bounded repeats of any size compile to BPG programs (not the host backtracker) whose
    native host twin -- and the Python twin on short lines -- give Java's find()."""
    rng = random.Random(gap)
    lines = _ctr_lines(rng, gap) + _lines(rng, 100)
    for p in CTR_PATS:
        d = N.compile_regex(p, 64, 4096)
        assert d["kind"] == 1 and d["bpg"], (p, d["error"])
        assert program_info(d["bpg"])["counters"] >= 1 and program_info(d["bpg"])["words"] <= 2, p
        rx = compile_java(p)
        for s in lines:
            if "+Z" in p and len(s) > 400:
                continue                    # (the oracle backtracks exponentially there)
            want = rx.search(s) is not None
            assert N.bpg_find(d["bpg"], s.encode()) == want, (p, len(s), s[:30])
            if len(s) < 200:
                assert run_program(d["bpg"], s.encode()) == want, (p, s)


@pytest.mark.gpu
@pytest.mark.parametrize("gap", [2100, 5000, 20000])
def test_counted_repeats_gpu_walks_match_host(gpu_device, gap):
    """The one-lane scan walk (k_bpg_scan) and the cooperative candidate walk (k_bpg_coop) keep the
    counts exactly as the host twin does, on lines longer than the bound."""
    lib = _lib(CTR_PATS)
    assert len(lib.bpg_regs) == len(CTR_PATS)
    lines = _ctr_lines(random.Random(gap + 1), gap)
    assert _scan(lib, lines, gpu_device) == _scan(lib, lines, torch.device("cpu"))
    text, ls, ll = _text_dev(lines, gpu_device)
    dfa = lib.device_tables(gpu_device)["dfa"]
    progs = {r: lib.bpg_program(r).tobytes() for r in lib.bpg_regs}
    cand = [(r << 32) | j for r in lib.bpg_regs for j in range(len(lines))]
    ct = torch.tensor(cand, dtype=torch.int64, device=gpu_device)
    N.bpg_cand_dev(ct.data_ptr(), ct.numel(), text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa,
                   torch.cuda.current_stream().cuda_stream)
    got = ct.cpu().tolist()
    for before, after in zip(cand, got):
        r, j = before >> 32, before & 0xFFFFFFFF
        assert (after >= 0) == N.bpg_find(progs[r], lines[j].encode()), (lib.regexes[r].pattern, len(lines[j]))


def test_lean_device_walk_bounds_and_parity_under_asan():
    """The DEVICE one-lane walks (bpg.h bpg_find_dev<W> and the lean one-word bpg_walk1) built for
    the host with AddressSanitizer (GPU ASan is unavailable): every program of the Java-shape test
    library plus Unicode / boundary-context / counted-repeat shapes in exact-size allocations, over
    padded text with non-ASCII code points and terminators -- no out-of-bounds read, and the same
    answer as the host twin bpg_find_w on every (program, line)."""
    import os
    import shutil
    import subprocess
    import sys
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "bpg_walk_check.py"), "--seed", "5", "--quick"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "mismatches 0" in r.stdout
