"""Pack Glushkov NFAs into 64-position groups for the MFMA state-transition kernel
(csrc/kernels/nfa_mfma.hip; table layout mirrored there)."""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

G_CLS, G_FIRST, G_LAST, G_REGMASK, G_F, G_META, G_CMASK, G_NULL, G_REGID, G_STRIDE = \
    0, 256, 271, 286, 294, 486, 487, 488, 496, 512
M = 64
CTX_ALL = 0x7FFF
NCTX = 15
MAX_REGS = 8


def _gated_conds(d) -> set:
    return {c for edges in d["nfa_follow"] for (_, c) in edges if c != CTX_ALL}


def fits_group(d) -> bool:
    """A byte-level Glushkov NFA (no code-point-only regex) of <= 64 positions, <= 2 gated conditions."""
    return 0 < d.get("npos", 0) <= M and "nfa_follow" in d and len(_gated_conds(d)) <= 2


def pack_groups(members: Sequence[Tuple[int, dict]]) -> List[List[Tuple[int, dict]]]:
    """Greedy first-fit: <= 64 positions, <= 8 regexes, <= 2 distinct gated edge conditions."""
    groups: List[List[Tuple[int, dict]]] = []
    state: List[Tuple[int, set]] = []
    for rid, d in members:
        gc = _gated_conds(d)
        for gi, (used, conds) in enumerate(state):
            if used + d["npos"] <= M and len(groups[gi]) < MAX_REGS and len(conds | gc) <= 2:
                groups[gi].append((rid, d))
                state[gi] = (used + d["npos"], conds | gc)
                break
        else:
            groups.append([(rid, d)])
            state.append((d["npos"], set(gc)))
    return groups


def build_group(members: Sequence[Tuple[int, dict]]) -> Tuple[np.ndarray, int]:
    tab = np.zeros(G_STRIDE, np.uint64)
    conds: List[int] = []
    base = 0
    for q, (rid, d) in enumerate(members):
        npos = d["npos"]
        cls = np.frombuffer(d["nfa_cls"], np.uint8).reshape(npos, 32)
        bits = np.unpackbits(cls, axis=1, bitorder="little")        # [npos, 256]
        for p in range(npos):
            m = np.uint64(1 << (base + p))
            tab[G_CLS + np.nonzero(bits[p])[0]] |= m
        for (p, c) in d["nfa_first"]:
            for ctx in range(NCTX):
                if (c >> ctx) & 1:
                    tab[G_FIRST + ctx] |= np.uint64(1 << (base + p))
        for (p, c) in d["nfa_last"]:
            for ctx in range(NCTX):
                if (c >> ctx) & 1:
                    tab[G_LAST + ctx] |= np.uint64(1 << (base + p))
        tab[G_REGMASK + q] = np.uint64(((1 << npos) - 1) << base)
        tab[G_NULL + q] = np.uint64(d["nfa_nullable"])
        tab[G_REGID + q] = np.uint64(rid)
        for p, edges in enumerate(d["nfa_follow"]):
            for (to, c) in edges:
                if c == CTX_ALL:
                    k = 0
                else:
                    if c not in conds:
                        conds.append(c)
                    k = 1 + conds.index(c)
                tab[G_F + 64 * k + base + p] |= np.uint64(1 << (base + to))
        base += npos
    assert base <= M and len(conds) <= 2 and len(members) <= MAX_REGS
    ncls = 1 + len(conds)
    tab[G_META] = np.uint64(ncls | (len(members) << 8))
    cm = (conds[0] if conds else 0) | ((conds[1] if len(conds) > 1 else 0) << 16)
    tab[G_CMASK] = np.uint64(cm)
    return tab, ncls
