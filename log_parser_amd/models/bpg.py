"""Bit-parallel Glushkov programs ("BPG") for regexes whose DFA blows up or that need code-point
boundary contexts.

A Glushkov NFA over CODE POINTS of M positions (one per character / class / property of the
regex: ``.``, ``[^é]`` or ``\\p{L}`` is one position) is simulated with the active-position set held
as W = ceil(M / 64) 64-bit words per line (W <= 32: bounded gaps up to ``X.{0,2000}Y``). The
reference's ``Pattern.compile(...).matcher(line).find()`` (``AnalysisService.java:62-65,93-95``;
secondaries ``ScoringService.java:315-347``) is exactly "does the NFA accept somewhere on the
line", so one pass over the line's code points answers it.

The program is built at library load by ``jregex.cpp`` ``bpg_program`` (exposed as the ``bpg``
bytes of ``N.compile_regex``), which decomposes the follow relation into word-parallel parts --
shift edges p -> p+1, self loops, spread fields (every active source reaches every target above
it: one multi-word subtraction for all fields), and exception rows -- and checks that the parts
rebuild every follow set. A bounded repeat of one class ``C{m,n}`` (n - m >= 16) is m plain
positions plus ONE counted position whose self loop holds while the youngest thread in it has
read fewer than n - m characters (``X.{0,20000}Y`` = 3 positions). Layout: ``csrc/kernels/bpg.h``. This module holds the pure-Python twin
of the walk (tests) and the header decoder.
"""
from __future__ import annotations

import bisect

import numpy as np

NCTX = 24
HDR_UNIFORM = 1 << 31
HDR_ANCHORED = 1 << 30
WIDTHS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32)   # word counts the device code is instantiated for
MAX_WORDS = 32


def program_info(prog) -> dict:
    prog = np.frombuffer(prog, np.uint64) if isinstance(prog, (bytes, bytearray)) else prog
    h = int(prog[0])
    return {"words": h & 0xFF, "exceptions": (h >> 8) & 0xFFF, "classes": (h >> 20) & 0x3FF,
            "uniform": bool(h & HDR_UNIFORM), "anchored": bool(h & HDR_ANCHORED),
            "unicode_word": bool((h >> 56) & 1), "ranges": int(prog[1]) & 0xFFFFFFFF,
            "counters": (h >> 57) & 7, "size": int(prog[1]) >> 32}


def _ascii_kind(c: int) -> int:
    if 48 <= c <= 57 or 65 <= c <= 90 or 97 <= c <= 122 or c == 95:
        return 2
    return 5 if c in (10, 13) else 3


def run_program(prog, line: bytes) -> bool:
    """Pure-Python twin of ``bpg_find_w`` (csrc/kernels/bpg.h): find() of one line."""
    prog = np.frombuffer(prog, np.uint64) if isinstance(prog, (bytes, bytearray)) else prog
    h = int(prog[0])
    W, E, ncls = h & 0xFF, (h >> 8) & 0xFFF, (h >> 20) & 0x3FF
    uniform, anchored = bool(h & HDR_UNIFORM), bool(h & HDR_ANCHORED)
    nullable = (h >> 32) & 0xFFFFFF
    nr = int(prog[1]) & 0xFFFFFFFF
    big = lambda ws: sum(int(x) << (64 * i) for i, x in enumerate(ws))  # noqa: E731
    o = 2
    shm, selfm, src, R, lo, hi = (big(prog[o + k * W:o + (k + 1) * W]) for k in range(6))
    o_first, o_last, o_amap = 2 + 6 * W, 2 + 30 * W, 2 + 54 * W
    o_cls = o_amap + 32
    o_exc = o_cls + ncls * W
    o_rng = o_exc + E * (W + 1)
    first = [big(prog[o_first + c * W:o_first + (c + 1) * W]) for c in range(NCTX)]
    last = [big(prog[o_last + c * W:o_last + (c + 1) * W]) for c in range(NCTX)]
    amap = prog[o_amap:o_amap + 32].view(np.uint16)
    cls = [big(prog[o_cls + k * W:o_cls + (k + 1) * W]) for k in range(ncls)]
    exc = []
    for e in range(E):
        x = int(prog[o_exc + e * (W + 1)])
        exc.append((x & 0xFFFF, (x >> 16) & 0xFFFFFF, big(prog[o_exc + e * (W + 1) + 1:o_exc + (e + 1) * (W + 1)])))
    rng = [int(x) for x in prog[o_rng:o_rng + nr]]
    # counted positions (bounded repeats of one class): [position, bound, youngest thread's count]
    ctr = [[int(x) & 0xFFFF, int(x) >> 16, 0] for x in prog[o_rng + nr:o_rng + nr + ((h >> 57) & 7)]]
    rlo = [x & 0x1FFFFF for x in rng]
    full = (1 << (64 * W)) - 1
    n = len(line)
    ft_len = 0
    if line.endswith(b"\r"):
        ft_len = 1
    elif line.endswith(b"\xc2\x85"):
        ft_len = 2
    elif line.endswith(b"\xe2\x80\xa8") or line.endswith(b"\xe2\x80\xa9"):
        ft_len = 3
    ft = n - ft_len if ft_len else -1

    def char(t):
        c = line[t]
        if c < 0x80:
            return int(amap[c]), _ascii_kind(c)
        k = 4 if c >= 0xF0 else 3 if c >= 0xE0 else 2
        b = [line[t + m] if t + m < n else 0x80 for m in range(1, 4)]
        if k == 2:
            cp = ((c & 31) << 6) | (b[0] & 63)
        elif k == 3:
            cp = ((c & 15) << 12) | ((b[0] & 63) << 6) | (b[1] & 63)
        else:
            cp = ((c & 7) << 18) | ((b[0] & 63) << 12) | ((b[1] & 63) << 6) | (b[2] & 63)
        e = rng[bisect.bisect_right(rlo, cp) - 1]
        kd = (e >> 37) & 3
        return (e >> 21) & 0xFFFF, 2 if kd == 1 else 5 if kd == 2 else 3

    def acc(S, ctx):
        return bool((nullable >> ctx) & 1) or bool(S & last[0 if uniform else ctx])

    S, prevk = 0, 0
    for t in range(n + 1):
        if t < n and 0x80 <= line[t] < 0xC0:
            continue                                   # inside a code point
        k, nk = char(t) if t < n else (0, 0)
        if t == ft and acc(S, prevk * 6 + 1):
            return True
        if acc(S, prevk * 6 + nk):
            return True
        if t == n:
            break
        ctx = prevk * 6 + nk
        Fo = (((S & shm) << 1) | (S & selfm)) & full
        t_ = (S & src) | hi
        dd = (t_ - lo) & full
        Fo |= R & ~(dd ^ t_) & full
        for p, cond, m in exc:
            if (S >> p) & 1 and (cond >> ctx) & 1:
                Fo |= m
        Fo |= first[0 if uniform else ctx]
        for c in ctr:                                  # entry -> count 1; stay while count < bound
            p, bound, cnt = c
            entry = (Fo >> p) & 1
            stay = (S >> p) & 1 and cnt < bound
            Fo |= stay << p
            c[2] = 1 if entry else min(cnt + 1, bound)
        S = Fo & cls[k]
        if anchored and not S:
            return False
        prevk = 1 if nk == 2 else 3 if nk == 5 else 2
    return False
