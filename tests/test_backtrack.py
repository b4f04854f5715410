"""Native Java-semantics backtracker (jregex BtRegex) for the regexes no automaton expresses:
backreferences, lookahead / lookbehind, atomic groups, possessive quantifiers, MULTILINE
anchors. Fuzzed against the javacompat oracle (Python ``regex`` with Java translation), then
end to end: a library with such patterns gives the golden model's events and scores, with the
device prefilter narrowing literal-bearing ones to candidate lines."""
import random

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from log_parser_amd import golden
from log_parser_amd.engine import Engine
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.models.schema import PatternSet
from log_parser_amd.native import N
from log_parser_amd.regex.javacompat import java_find
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_log

ATOMS = ["a", "b", "c", "A", " ", "1", ".", r"\d", r"\w", r"\s", "[ab]", "[^a]", r"\b", "^", "$", "é"]


def _rx(rng, depth, ngroups):
    parts = []
    for _ in range(rng.randint(1, 4)):
        r = rng.random()
        if r < 0.12 and depth < 2:
            ngroups[0] += 1
            a = "(" + "|".join(_rx(rng, depth + 1, ngroups) for _ in range(rng.randint(1, 2))) + ")"
        elif r < 0.2 and ngroups[0]:
            a = "\\" + str(rng.randint(1, ngroups[0]))
        elif r < 0.28 and depth < 2:
            kind = rng.choice(["?=", "?!", "?<=", "?<!", "?>"])
            inner = "".join(rng.choice(["a", "b", r"\d", "[ab]", " "]) for _ in range(rng.randint(1, 2)))
            a = f"({kind}{inner})" if kind.startswith("?<") else f"({kind}{_rx(rng, depth + 1, ngroups)})"
        else:
            a = rng.choice(ATOMS)
        if a not in ("^", "$", r"\b") and not a.startswith("(?") and not a.startswith("\\") or a in (r"\d", r"\w", r"\s"):
            q = rng.random()
            if q < 0.12:
                a += rng.choice(["*", "*?", "*+"])
            elif q < 0.22:
                a += rng.choice(["+", "+?", "++"])
            elif q < 0.3:
                a += rng.choice(["?", "??", "?+"])
        parts.append(a)
    return "".join(parts)


def _line(rng):
    return "".join(rng.choice("abcAB 1.é\t") for _ in range(rng.randint(0, 14))) + ("\r" if rng.random() < 0.1 else "")


@settings(max_examples=400, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
@given(st.integers(min_value=0, max_value=2**31 - 1))
def test_backtracker_matches_java_oracle(seed):
    rng = random.Random(seed)
    pat = _rx(rng, 0, [0])
    if rng.random() < 0.15:
        pat = "(?i)" + pat
    bt = N.BtSet([pat])
    if not bt.ok(0):
        return
    for _ in range(25):
        line = _line(rng)
        try:
            want = java_find(pat, line)
        except Exception:
            return
        assert bt.find(0, line) == want, (pat, line)


@pytest.mark.parametrize("pat,line,want", [
    (r"(a)\1", "xaay", True), (r"(?<=ab)c", "abc", True), (r"(?<!ab)c", "abc", False), (r"a*+a", "aaaa", False),
    (r"(?>a*?)a", "aaa", True), (r"(?i)(ab)\1", "abAB", True), (r"(?m)^b", "a\rb", True), (r"(?m)^", "", False),
    (r"(?<n>x+)\k<n>", "xxxx", True), (r"(x*)*y", "x" * 40 + "z", False), (r"\b(\w+) \1\b", "the the cat", True),
    # '.' takes a whole code point: backtracking must not split 'é' (two UTF-8 bytes)
    (r"1+\w?+.(?!c.\w)", "baaA .1écbBB", False), (r".(?!\w)", "é", True), (r"^.{2}$", "éa", True),
    # an empty loop iteration ends the loop but keeps its captures (Java Loop / LazyLoop)
    (r"([ab]a|(?<=[ab]))*? \1.", "abABa \tc\t cB", True), (r"(a?)*b\1", "b", True),
])
def test_backtracker_java_cases(pat, line, want):
    assert N.BtSet([pat]).find(0, line) == want


def test_backtracker_classification():
    d = N.compile_regex(r"(\w+) failed: \1")
    assert d["kind"] == 2 and d["bt_ok"] and d["literals"] == [b" failed: "]
    assert N.compile_regex(r"(?<=a*)b")["kind"] == 3               # Java: no obvious maximum length
    assert N.compile_regex(r"\p{InGreek}")["kind"] == 0           # unicode blocks: a byte DFA
    assert N.BtSet([r"(\p{InGreek})\1"]).find(0, "xΣΣ")          # ... and in the backtracker


def _library():
    regexes = [r"(\w+)Aux0 \1", r"(?i)fatal (?=\w+Failure)", r"(?<!WARN )\[app\] (\w+)Step0", r"\b(\w)\w*\1Failure\b",
               r"(?>\d+)Step", r"timed?+ out", r"^(?:(?!INFO).)*Aux1\b", r"(\w)\1{3,}"]
    pats = [{"id": f"bt{i}", "name": rx, "severity": "HIGH", "primary_pattern": {"regex": rx, "confidence": 0.7},
             "context_extraction": {"lines_before": 2, "lines_after": 1}} for i, rx in enumerate(regexes)]
    from log_parser_amd.utils.synth import make_library
    sets, trig = make_library(40, seed=17)
    sets.append(PatternSet.model_validate({"metadata": {"library_id": "bt"}, "patterns": pats}))
    return sets, trig


def test_engine_with_backtracking_regexes_matches_golden():
    p = ScoringParams()
    sets, trig = _library()
    lib = CompiledLibrary(sets, p)
    s = lib.summary()
    assert s["host_fallback"] >= 6 and s["host_backtracker"] == s["host_fallback"]
    assert any(lits for _, _, lits in lib.host_plan) and any(not lits for _, _, lits in lib.host_plan)
    logs = make_log(3000, trig, seed=18, hit_rate=0.1, crlf_rate=0.05)
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    r = eng.analyze(logs)
    g = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in r["events"]] == \
        [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
    assert sum(e["matchedPattern"]["id"].startswith("bt") for e in r["events"]) > 20
    np.testing.assert_allclose([e["score"] for e in r["events"]], [e["score"] for e in g["events"]], rtol=1e-12)


@pytest.mark.gpu
def test_engine_with_backtracking_regexes_gpu(gpu_device):
    p = ScoringParams()
    sets, trig = _library()
    lib = CompiledLibrary(sets, p)
    logs = make_log(3000, trig, seed=19, hit_rate=0.1)
    eng = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device)}), device=gpu_device)
    r = eng.analyze(logs)
    g = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in r["events"]] == \
        [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
    np.testing.assert_allclose([e["score"] for e in r["events"]], [e["score"] for e in g["events"]], rtol=1e-12)


@pytest.mark.gpu
def test_backref_pattern_cost_on_a_million_lines(gpu_device):
    """One literal-bearing backreference pattern over 1M lines: the device prefilter narrows it
    to candidate lines, so the host backtracker adds little (AnalysisService.java:64,95)."""
    import time
    from log_parser_amd.ops import kernels as K
    p = ScoringParams()
    sets, trig = _library()
    base = CompiledLibrary(sets[:-1], p)
    one = PatternSet.model_validate({"metadata": {"library_id": "bt"}, "patterns": [
        {"id": "br", "name": "br", "severity": "HIGH", "primary_pattern": {"regex": r"(\w+)Aux0 \1", "confidence": 0.7}}]})
    lib = CompiledLibrary(sets[:-1] + [one], p)
    block = make_log(100_000, trig, seed=20, hit_rate=0.01).encode()
    data = block * 10
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(gpu_device)
    ls, ll = K.split_lines(t, len(data))
    host = np.frombuffer(data, np.uint8)
    times = {}
    for name, L in (("base", base), ("backref", lib)):
        e = Engine(L, Config.load(overrides={"engine.device": str(gpu_device)}), device=gpu_device)
        for _ in range(2):
            e.match_hits(t, len(data), ls, ll, host_text=host)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            e.match_hits(t, len(data), ls, ll, host_text=host)
        torch.cuda.synchronize()
        times[name] = (time.perf_counter() - t0) / 3
    print("1M lines, one backref pattern:", times)
    assert times["backref"] - times["base"] < 0.1


@pytest.mark.gpu
def test_host_regex_side_path_without_host_bytes(gpu_device):
    """Without host bytes the side path copies the text to the host once: same hits as with the
    caller's host copy."""
    from log_parser_amd.ops import kernels as K
    p = ScoringParams()
    sets, trig = _library()
    # literal-bearing host regexes only (a literal-free one needs every line on the host)
    lits = [rx for rx in (r"(\w+)Aux0 \1", r"(?i)fatal (?=\w+Failure)", r"(?>\d+)Step", r"timed?+ out")]
    from log_parser_amd.models.schema import PatternSet as PS
    extra = PS.model_validate({"metadata": {"library_id": "bt2"}, "patterns": [
        {"id": f"h{i}", "name": rx, "severity": "LOW", "primary_pattern": {"regex": rx, "confidence": 0.5}}
        for i, rx in enumerate(lits)]})
    lib = CompiledLibrary(sets[:-1] + [extra], p)
    assert lib.host_plan and all(lits for _, _, lits in lib.host_plan)
    data = make_log(20000, trig, seed=21, hit_rate=0.05).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(gpu_device)
    ls, ll = K.split_lines(t, len(data))
    e = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device)}), device=gpu_device)
    a = e.match_hits(t, len(data), ls, ll, host_text=np.frombuffer(data, np.uint8)).cpu()
    b = e.match_hits(t, len(data), ls, ll, host_text=None).cpu()
    assert torch.equal(a, b)
    hr = torch.tensor(lib.host_regs)
    assert bool(torch.isin(a >> 32, hr).any())


def _bt_library(n_bt=6):
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.utils.config import ScoringParams
    from log_parser_amd.utils.synth import backtracker_patterns, make_library
    sets, trig = make_library(40, seed=71, sequence_rate=0.5)
    ps, bt_trig = backtracker_patterns(n_bt, seed=3)
    return sets + [ps], trig + bt_trig, CompiledLibrary(sets + [ps], ScoringParams())


def test_relaxation_is_a_superset_and_device_fed():
    """Every backtracker shape of the bench gets a regular relaxation (a DFA / BPG program on the
    device), whose find() holds wherever the Java-semantics original's does -- so the candidate
    lines the device hands the host never miss a match."""
    import random
    from log_parser_amd.native import N
    from log_parser_amd.regex.javacompat import compile_java
    sets, trig, lib = _bt_library(8)
    assert len(lib.host_dev) == 8 and not lib.host_plan_undev
    pats = [p.primary_pattern.regex for p in sets[-1].patterns] + [
        r"(\w+)Aux0 \1", r"^(\w*)\1$", r"(?i)fatal (?=\w+Failure)", r"(?<!INFO )ERROR\b", r"(?>a+)b", r"x++y",
        r"(?i)(ab)\1", r"(?m)^ERR(?=\w)", r"(?<=id=)(\d+) .* \1"]
    rng = random.Random(5)
    toks = ["ab", "AB", "a", "b", "z", "x", "y", "123", "-", "415-8812-8812-415", "ERROR", "INFO ", "fatal ",
            "FooFailure", "Aux0", "id=", "7", " ", "é"] + [t["sample"] for t in trig[-8:]]
    lines = ["".join(rng.choice(toks) for _ in range(rng.randint(0, 10))) for _ in range(4000)]
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.models.schema import PatternSet
    from log_parser_amd.utils.config import ScoringParams
    relaxed = CompiledLibrary([PatternSet.model_validate({"metadata": {"library_id": "r"}, "patterns": [
        {"id": f"r{i}", "name": p, "severity": "LOW", "primary_pattern": {"regex": "(?#relax)" + p, "confidence": 0.5}}
        for i, p in enumerate(pats)]})], ScoringParams())
    from log_parser_amd.engine import Engine
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.config import Config
    for p in pats:
        d = N.compile_regex("(?#relax)" + p, 2048, 4096)
        assert d["kind"] in (0, 1), (p, d["error"])
    eng = Engine(relaxed, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    blob = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(blob)), dtype=torch.uint8)
    t[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(blob))
    hits = set(eng.match_hits(t, len(blob), ls, ll).tolist())
    n_orig = 0
    for i, p in enumerate(pats):
        rx = compile_java(p)
        r = int(relaxed.primary_reg[i])
        for j, s in enumerate(lines):
            if rx.search(s) is not None:
                n_orig += 1
                assert (r << 32 | j) in hits, (p, s)
    assert n_orig > 200


@pytest.mark.gpu
def test_device_fed_backtracker_bulk_step_equals_cpu(gpu_device):
    """The bulk step with backtracker primaries: their relaxed automata find candidate lines on the
    GPU, k_take_host exports them, the host checks them while the step stays queued, k_wait_host
    appends the verified keys -- events and scores equal the CPU engine's (host side path)."""
    from log_parser_amd.engine import Engine, Segments
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.parallel.dp import ShardedAnalyzer
    from log_parser_amd.utils.config import Config
    from log_parser_amd.utils.synth import make_log
    sets, trig, lib = _bt_library(6)
    logs = make_log(30000, trig, seed=72, hit_rate=0.06)
    data = logs.encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    cpu = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    ls, ll = K.split_lines(t, len(data))
    ref = cpu.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), cpu.freq_carry(),
                  host_text=np.frombuffer(data, np.uint8))
    bt_ids = {lib.patterns.index(p) for p in sets[-1].patterns}
    assert sum(int(x) in bt_ids for x in ref.ev_pat.numpy()) >= 20
    eng = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device)}), device=gpu_device)
    sa = ShardedAnalyzer(eng)
    for _ in range(3):                    # repeated steps: sequence numbers, reused export buffers
        out = sa.step(t.to(gpu_device), len(data), None, None, 0, 0, topk=5, host_text=np.frombuffer(data, np.uint8))
        r = out.result
        np.testing.assert_array_equal(r.ev_line.cpu().numpy(), ref.ev_line.numpy())
        np.testing.assert_array_equal(r.ev_pat.cpu().numpy(), ref.ev_pat.numpy())
    assert eng._host_side is not None and eng._host_side.seq >= 3


@pytest.mark.gpu
def test_side_path_gpu_wait_timeout_falls_back_to_host_verified_path(gpu_device):
    """A host verification slower than the GPU's wait (here: a 0.1 us wait, so every device-fed
    attempt times out) does not loop through the same timeout: the step re-runs once on the
    host-verified path and its events equal the CPU engine's; superseded regions are freed."""
    from log_parser_amd.engine import Engine, Segments
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.parallel.dp import ShardedAnalyzer
    from log_parser_amd.utils.config import Config
    from log_parser_amd.utils.synth import make_log
    sets, trig, lib = _bt_library(6)
    data = make_log(20000, trig, seed=73, hit_rate=0.06).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    cpu = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    ls, ll = K.split_lines(t, len(data))
    ref = cpu.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), cpu.freq_carry(),
                  host_text=np.frombuffer(data, np.uint8))
    eng = Engine(lib, Config.load(overrides={"engine.device": str(gpu_device), "engine.side-path-wait-s": 1e-7}),
                 device=gpu_device)
    sa = ShardedAnalyzer(eng)
    for _ in range(3):
        out = sa.step(t.to(gpu_device), len(data), None, None, 0, 0, topk=5, host_text=np.frombuffer(data, np.uint8))
        np.testing.assert_array_equal(out.result.ev_line.cpu().numpy(), ref.ev_line.numpy())
        np.testing.assert_array_equal(out.result.ev_pat.cpu().numpy(), ref.ev_pat.numpy())
    hs = eng._host_side
    assert hs.fallbacks >= 1 and hs.waits_failed >= hs.fallbacks
    hs.close()
    assert not hs._retired


def test_native_side_worker_verifies_exported_candidates():
    """bind.cpp SideWorker (the side path's native host half) on plain host memory: it waits for
    the export's sequence word, checks each exported candidate line with the backtracker and
    publishes (verified keys, count, then sequence); an export larger than the buffer publishes -1
    and asks for a bigger one."""
    import time
    sets, trig, lib = _bt_library(4)
    text = "\n".join(t["sample"] for t in trig[-4:]) + "\nno match here\n" + trig[-4]["sample"].upper() + "\n"
    data = np.frombuffer(text.encode(), np.uint8).copy()
    lines = text.encode().split(b"\n")[:-1]
    starts = np.cumsum([0] + [len(x) + 1 for x in lines[:-1]])
    w = N.SideWorker(lib.host_bt, [int(x) for x in lib.host_local])
    cap = 64
    out = np.zeros(3 * cap + 2, np.int64)
    inb = np.zeros(cap + 3, np.int64)
    keys = [(r << 32) | x for x in range(len(lines)) for r in lib.host_dev]
    n = len(keys)
    out[:n] = keys
    out[cap:cap + n] = [starts[k & 0xFFFFFFFF] for k in keys]
    out[2 * cap:2 * cap + n] = [len(lines[k & 0xFFFFFFFF]) for k in keys]

    def wait(seq):
        t0 = time.time()
        while inb[cap + 1] != seq:
            assert time.time() - t0 < 10
            time.sleep(0.001)

    w.submit(1, data.ctypes.data, cap, out.ctypes.data, 0, inb.ctypes.data)
    time.sleep(0.01)                       # the worker polls until the export is published
    out[3 * cap], out[3 * cap + 1] = n, 1
    wait(1)
    got = sorted(inb[:inb[cap]].tolist())
    want = sorted(k for k in keys if lib.host_bt.find(int(lib.host_local[k >> 32]),
                                                      lines[k & 0xFFFFFFFF].decode()))
    assert got == want and len(want) >= 4 and w.take_error() == ""
    # two regions (prefilter candidates, then scan keys): the answer covers both
    out_b = np.zeros(3 * cap + 2, np.int64)
    h = n // 2
    out_b[:n - h], out_b[cap:cap + n - h], out_b[2 * cap:2 * cap + n - h] = \
        out[h:n], out[cap + h:cap + n], out[2 * cap + h:2 * cap + n]
    w.submit(2, data.ctypes.data, cap, out.ctypes.data, out_b.ctypes.data, inb.ctypes.data)
    out[3 * cap], out[3 * cap + 1] = h, 2
    time.sleep(0.01)
    assert inb[cap + 1] != 2                # still waiting for region B
    out_b[3 * cap], out_b[3 * cap + 1] = n - h, 2
    wait(2)
    assert sorted(inb[:inb[cap]].tolist()) == want
    out[3 * cap], out[3 * cap + 1] = cap + 5, 3     # an export that overflowed its buffer
    w.submit(3, data.ctypes.data, cap, out.ctypes.data, 0, inb.ctypes.data)
    wait(3)
    assert inb[cap] == -1 and w.need == cap + 5
