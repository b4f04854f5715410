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
