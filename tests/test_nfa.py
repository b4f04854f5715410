"""NFA (MFMA state-transition kernel / host twin) vs the DFA engine and the golden oracle."""
import random

import numpy as np
import pytest
import torch

from log_parser_amd.golden import CONTEXT_REGEXES
from log_parser_amd.models.nfa import build_group, pack_groups
from log_parser_amd.native import N
from log_parser_amd.ops import kernels as K
from log_parser_amd.regex.javacompat import java_find

PATS = [r"(a|b)*a(a|b){6}", r"\bfoo\b.*bar", r"x\By", r"^\s*at\s+[\w.]+\(", r"(?i)warn(ing)?\b", r"[^a]b$",
        r"é+z", r"colou?r", r"\d{2,4}-\d+", r"(ab|a)(bc|c)", r"a\b b", r"q\Bq"]


def _lines(rng, n):
    alpha = "abfoqxyzr -é\t0123456789WARNINGwarn()"
    out = []
    for _ in range(n):
        s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 40)))
        if rng.random() < 0.1:
            s += "\r"
        out.append(s)
    out += ["foo bar", "  at com.x.Y(", "WARNING x", "colour", "12-345", "abc", "a b", "qq", "éééz", "xb"]
    return out


def _run(members, lines, dev):
    tabs, ncls = zip(*[build_group(g) for g in members])
    blob = "\n".join(lines).encode()
    t = torch.zeros(K.padded_len(len(blob)), dtype=torch.uint8)
    t[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    starts, lens, pos = [], [], 0
    for l in lines:
        b = len(l.encode())
        starts.append(pos)
        lens.append(b)
        pos += b + 1
    ls = torch.tensor(starts, dtype=torch.int64)
    ll = torch.tensor(lens, dtype=torch.int32)
    g = torch.from_numpy(np.concatenate(tabs).view(np.int64))
    out = []
    for k in sorted(set(ncls)):
        gl = torch.tensor([i for i, c in enumerate(ncls) if c == k], dtype=torch.int32)
        out.append(K.nfa_scan(g.to(dev), gl.to(dev), k, t.to(dev), ls.to(dev), ll.to(dev), 4096).cpu())
    return set(torch.cat(out).tolist())


@pytest.mark.parametrize("seed", [0, 1])
def test_nfa_host_equals_oracle(seed):
    rng = random.Random(seed)
    lines = _lines(rng, 300)
    members = [(i, N.compile_regex(p, 64, 4096)) for i, p in enumerate(PATS)]
    groups = pack_groups(members)
    got = _run(groups, lines, torch.device("cpu"))
    want = {(i << 32) | j for i, p in enumerate(PATS) for j, l in enumerate(lines) if java_find(p, l)}
    assert got == want


def test_context_groups_fit():
    """The 4 context regexes pack into at most two 64-position MFMA groups (the exact UTF-8 '.' of
    the stack-frame regex costs ~10 byte positions); each group ORs its members' feature bits."""
    members = [(i, N.compile_regex(p)) for i, p in enumerate(CONTEXT_REGEXES)]
    groups = pack_groups(members)
    assert 1 <= len(groups) <= 2
    for g in groups:
        build_group(g)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3])
def test_nfa_mfma_gpu_equals_host(gpu_device, seed):
    rng = random.Random(seed)
    lines = _lines(rng, 2000)
    members = [(i, N.compile_regex(p, 64, 4096)) for i, p in enumerate(PATS)]
    groups = pack_groups(members)
    assert _run(groups, lines, gpu_device) == _run(groups, lines, torch.device("cpu"))


# ---- engine.nfa-engine=mfma end to end: the MFMA engine serving regexes whose DFA is refused
MFMA_PATS = [r"error.{0,12}timeout", r"(a|b)*a(a|b){5}x", r"\bconn(ection)? (reset|refused).{0,9}port \d+",
             r"(?i)fail(ed|ure)?.{0,8}retry \d", r"[A-Z]{2}\d{2,5}(-[a-z]+){1,3}\b"]


def _mfma_engine(dev):
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.models.schema import PatternSet
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_library
    sets, trig = make_library(30, seed=12)
    pats = [{"id": f"m{i}", "name": rx, "severity": "HIGH", "primary_pattern": {"regex": rx, "confidence": 0.8},
             "context_extraction": {"lines_before": 1, "lines_after": 1}} for i, rx in enumerate(MFMA_PATS)]
    sets.append(PatternSet.model_validate({"metadata": {"library_id": "mfma"}, "patterns": pats}))
    p = ScoringParams()
    # a small DFA budget sends the gap / counted shapes to the NFA engines; mfma serves them
    lib = CompiledLibrary(sets, p, max_dfa_states=24, nfa_engine="mfma")
    eng = Engine(lib, Config.load(overrides={"engine.device": str(dev), "engine.nfa-engine": "mfma"}), device=dev)
    return eng, lib, sets, trig, p


def _mfma_docs(trig, seed):
    from log_parser_amd.utils.synth import make_log
    extra = ["error while waiting: timeout", "connection refused by peer port 8080", "FAILED twice, retry 3",
             "AB1234-foo-bar ok", "abababaabbbabx", "error.....................timeout"]
    rng = random.Random(seed)
    docs = []
    for k in range(3):
        lines = make_log(600 + 200 * k, trig, seed=seed + k, hit_rate=0.1).split("\n")
        for _ in range(40):
            lines.insert(rng.randrange(len(lines)), rng.choice(extra))
        docs.append("\n".join(lines))
    return docs


def _check_mfma(dev):
    import json
    from log_parser_amd import golden
    eng, lib, sets, trig, p = _mfma_engine(dev)
    assert lib.summary()["nfa_mfma"] >= len(MFMA_PATS)
    docs = _mfma_docs(trig, 5)
    outs = [json.loads(o) for o in eng.analyze_batch_json(docs)]
    ft = golden.FrequencyTracker(p)
    got_m = 0
    for o, d in zip(outs, docs):
        g = golden.analyze(d, sets, p, ft)
        assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
            [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
        np.testing.assert_allclose([e["score"] for e in o["events"]], [e["score"] for e in g["events"]], rtol=1e-12)
        got_m += sum(e["matchedPattern"]["id"].startswith("m") for e in o["events"])
    assert got_m > 20
    return eng


def test_engine_nfa_mfma_end_to_end_cpu():
    """engine.nfa-engine=mfma through the whole engine (host twin of the MFMA kernel) == golden."""
    _check_mfma(torch.device("cpu"))


@pytest.mark.gpu
def test_engine_nfa_mfma_end_to_end_gpu(gpu_device):
    """The same on the GPU: the NFA regexes are matched by the MFMA state-transition kernel
    (k_nfa_* on matrix cores) inside the engine's match stage, results == golden (rtol 1e-12)."""
    eng = _check_mfma(gpu_device)
    assert any(g.numel() for g in eng.tabs["nfa_scan_lists"].values())
