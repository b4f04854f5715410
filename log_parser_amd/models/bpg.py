"""Bit-parallel Glushkov programs ("BPG") for regexes whose DFA blows up.

A Glushkov NFA of M positions (``jregex`` output: per-position byte classes, follow edges with
boundary-context conditions, first / last sets) is simulated with the active-position set held as
W = ceil(M / 64) 64-bit words per line. The reference's ``Pattern.compile(...).matcher(line).find()``
(``AnalysisService.java:62-65,93-95``; secondaries ``ScoringService.java:315-347``) is exactly "does
the NFA accept somewhere on the line", so one pass over the line answers it.

The transition ``S' = (Follow(S) | first[ctx]) & cls[byte]`` is evaluated from a *decomposition* of
the follow relation found at library load, so the common log-regex shapes cost O(W) word
operations per byte instead of O(M) table lookups:

* **shift** edges p -> p+1 (concatenation): ``(S & shm) << 1`` with the carry across words;
* **self** edges p -> p (``x*`` / ``x+``, UTF-8 continuation loops of ``.``): ``S & selfm``;
* **spread fields**: a position range [lo, hi] with target mask R and source mask Src such that every
  source p reaches every target above it (the nested-optional structure Glushkov gives bounded gaps
  ``X.{0,120}Y`` and optional runs): all fields at once with ONE multi-word subtraction
  (``d = (S & Src | Hi) - Lo``; targets above the lowest active source = ``R & ~(d ^ (S & Src | Hi))``;
  the guard bit Hi stops every borrow inside its field);
* **exceptions**: every remaining edge (loop-backs of repeated groups, boundary-gated edges) as
  (source, condition, target mask) entries, ORed in when the source is active.

The decomposition is exact: every position's follow set is rebuilt from the parts and compared.
Program layout (uint64 words; mirrored by ``csrc/kernels/bpg.h``)::

    [0]   header: W | E << 8 | ncls << 20 | anchored << 30 | uniform << 31 | nullable-context mask << 32
    shm[W] selfm[W] src[W] R[W] lo[W] hi[W]
    first[15][W] last[15][W]        (per boundary context; uniform -> only [0] is read)
    bytemap[32]                     (256 bytes: byte -> class)
    cls[ncls][W]
    exc[E][1 + W]                   (src | cond << 16, then the target mask)
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

CTX_ALL = 0x7FFF
NCTX = 15
MAX_WORDS = 8            # 512 positions (csrc/kernels/bpg.h BPG_MAX_W)
MAX_EXC = 256
HDR_UNIFORM = 1 << 31
HDR_ANCHORED = 1 << 30
WIDTHS = (1, 2, 3, 4, 6, 8)   # word counts the device code is instantiated for (bpg.h bpg_find)


def _mask_words(bits: Sequence[int], W: int) -> np.ndarray:
    m = np.zeros(W, np.uint64)
    for b in bits:
        m[b >> 6] |= np.uint64(1 << (b & 63))
    return m


def decompose(npos: int, follow: Sequence[Sequence[Tuple[int, int]]]):
    """Glushkov follow relation -> (shift set, self set, fields [(lo, hi, R, Src)], exceptions
    {src: [(cond, targets)]}). Exact: the parts rebuild every follow set."""
    F: List[set] = [set() for _ in range(npos)]
    gated: Dict[Tuple[int, int], set] = {}
    for p, edges in enumerate(follow):
        for to, c in edges:
            if c == CTX_ALL:
                F[p].add(to)
            else:
                gated.setdefault((p, c), set()).add(to)
    shift = {p for p in range(npos) if p + 1 in F[p]}
    selfl = {p for p in range(npos) if p in F[p]}
    covered: List[set] = [set() for _ in range(npos)]
    for p in shift:
        covered[p].add(p + 1)
    for p in selfl:
        covered[p].add(p)
    fields = []
    p = 0
    while p < npos:
        rest = F[p] - covered[p]
        fwd = {q for q in rest if q > p}
        if not fwd:
            p += 1
            continue
        R = {q for q in F[p] if q > p}
        hi = max(R)
        # targets reached by later sources too (a field grows while its sources reach further)
        src = [s for s in range(p, hi + 1) if {q for q in R if q > s} <= F[s]]
        if hi - p >= 1 and len(R) >= 2:
            fields.append((p, hi, sorted(R), src))
            for s in src:
                covered[s] |= {q for q in R if q > s}
            p = hi + 1
        else:
            p += 1
    exc: Dict[int, List[Tuple[int, set]]] = {}
    for p in range(npos):
        rest = F[p] - covered[p]
        if rest:
            exc.setdefault(p, []).append((CTX_ALL, rest))
    for (p, c), tos in gated.items():
        exc.setdefault(p, []).append((c, tos))
    # exactness check
    for p in range(npos):
        rebuilt = set(covered[p])
        for c, tos in exc.get(p, []):
            if c == CTX_ALL:
                rebuilt |= tos
        assert rebuilt == F[p], (p, rebuilt ^ F[p])
    return shift, selfl, fields, exc


def build_program(d: dict) -> Optional[np.ndarray]:
    """jregex ``compile_regex`` dict of an automaton regex -> BPG program (uint64), or None when
    it does not fit (more than MAX_WORDS words or MAX_EXC exception entries)."""
    npos = int(d.get("npos", 0))
    if npos <= 0:
        return None
    need = (npos + 63) // 64
    if need > MAX_WORDS:
        return None
    W = next(w for w in WIDTHS if w >= need)
    shift, selfl, fields, exc = decompose(npos, d["nfa_follow"])
    n_exc = sum(len(v) for v in exc.values())
    if n_exc > MAX_EXC:
        return None
    cls_bits = np.unpackbits(np.frombuffer(d["nfa_cls"], np.uint8).reshape(npos, 32), axis=1,
                             bitorder="little").astype(bool)          # [npos, 256]
    # byte classes: distinct columns
    cols: Dict[bytes, int] = {}
    bytemap = np.zeros(256, np.uint8)
    reps: List[np.ndarray] = []
    for b in range(256):
        key = np.packbits(cls_bits[:, b]).tobytes()
        k = cols.get(key)
        if k is None:
            k = cols[key] = len(reps)
            reps.append(np.flatnonzero(cls_bits[:, b]))
        bytemap[b] = k
    ncls = len(reps)
    first = np.zeros((NCTX, W), np.uint64)
    last = np.zeros((NCTX, W), np.uint64)
    for tab, lst in ((first, d["nfa_first"]), (last, d["nfa_last"])):
        for p, c in lst:
            for ctx in range(NCTX):
                if (c >> ctx) & 1:
                    tab[ctx, p >> 6] |= np.uint64(1 << (p & 63))
    uniform = bool((first == first[0]).all() and (last == last[0]).all())
    nullable = int(d["nfa_nullable"]) & CTX_ALL
    # first set only after BOS (prev kind 0 = contexts 0..4): once the state empties, nothing matches
    anchored = not first[5:].any() and not (nullable >> 5)
    hdr = (W | (n_exc << 8) | (ncls << 20) | (HDR_UNIFORM if uniform else 0) | (HDR_ANCHORED if anchored else 0)
           | (nullable << 32))
    R_all, src_all, lo_all, hi_all = set(), set(), set(), set()
    for lo, hi, R, src in fields:
        R_all |= set(R)
        src_all |= set(src)
        lo_all.add(lo)
        hi_all.add(hi)
    parts = [np.array([hdr], np.uint64),
             _mask_words(shift, W), _mask_words(selfl, W), _mask_words(src_all, W), _mask_words(R_all, W),
             _mask_words(lo_all, W), _mask_words(hi_all, W), first.reshape(-1), last.reshape(-1),
             bytemap.view(np.uint64)]
    for r in reps:
        parts.append(_mask_words(r, W))
    for p in sorted(exc):
        for c, tos in exc[p]:
            parts.append(np.array([p | (c << 16)], np.uint64))
            parts.append(_mask_words(tos, W))
    return np.concatenate(parts)


def program_info(prog: np.ndarray) -> dict:
    h = int(prog[0])
    return {"words": h & 0xFF, "exceptions": (h >> 8) & 0xFFF, "classes": (h >> 20) & 0x3FF,
            "uniform": bool(h & HDR_UNIFORM), "anchored": bool(h & HDR_ANCHORED), "size": int(prog.size)}


def run_program(prog: np.ndarray, line: bytes) -> bool:
    """Pure-Python twin of ``bpg_find`` (csrc/kernels/bpg.h) for tests: find() of one line."""
    h = int(prog[0])
    W, E, ncls = h & 0xFF, (h >> 8) & 0xFFF, (h >> 20) & 0x3FF
    uniform, nullable = bool(h & HDR_UNIFORM), (h >> 32) & CTX_ALL
    anchored = bool(h & HDR_ANCHORED)
    big = lambda ws: sum(int(x) << (64 * i) for i, x in enumerate(ws))  # noqa: E731
    o = 1
    shm, selfm, src, R, lo, hi = (big(prog[o + k * W:o + (k + 1) * W]) for k in range(6))
    o += 6 * W
    first = [big(prog[o + c * W:o + (c + 1) * W]) for c in range(NCTX)]
    o += NCTX * W
    last = [big(prog[o + c * W:o + (c + 1) * W]) for c in range(NCTX)]
    o += NCTX * W
    bm = prog[o:o + 32].view(np.uint8)
    o += 32
    cls = [big(prog[o + k * W:o + (k + 1) * W]) for k in range(ncls)]
    o += ncls * W
    exc = []
    for _ in range(E):
        e = int(prog[o])
        exc.append((e & 0xFFFF, (e >> 16) & 0xFFFF, big(prog[o + 1:o + 1 + W])))
        o += 1 + W
    full = (1 << (64 * W)) - 1
    ft_len = 0
    if line.endswith(b"\r"):
        ft_len = 1
    elif line.endswith(b"\xc2\x85"):
        ft_len = 2
    elif line.endswith(b"\xe2\x80\xa8") or line.endswith(b"\xe2\x80\xa9"):
        ft_len = 3
    ft = len(line) - ft_len if ft_len else -1

    def kind(c):
        if c < 0:
            return 0
        w = (48 <= c <= 57) or (65 <= c <= 90) or (97 <= c <= 122) or c == 95
        return 2 if w else (4 if 0x80 <= c <= 0xBF else 3)

    def acc(S, ctx):
        return bool((nullable >> ctx) & 1) or bool(S & last[0 if uniform else ctx])

    S, prevk = 0, 0
    for t in range(len(line) + 1):
        c = line[t] if t < len(line) else -1
        nk = kind(c)
        if t == ft and acc(S, prevk * 5 + 1):
            return True
        if acc(S, prevk * 5 + nk):
            return True
        if t == len(line):
            break
        ctx = prevk * 5 + nk
        Fo = (((S & shm) << 1) | (S & selfm)) & full
        t_ = (S & src) | hi
        dd = (t_ - lo) & full
        Fo |= R & ~(dd ^ t_) & full
        for p, cond, m in exc:
            if (S >> p) & 1 and (cond >> ctx) & 1:
                Fo |= m
        S = (Fo | first[0 if uniform else ctx]) & cls[int(bm[c])]
        if anchored and not S:
            return False
        prevk = 1 if nk == 2 else 2
    return False
