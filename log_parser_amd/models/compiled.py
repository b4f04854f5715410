"""Pattern library -> immutable device tables (compiled once at load, never per request).

The reference recompiles every primary / secondary / sequence regex on every request and
stores the compiled object on shared singletons (``AnalysisService.java:55-86``; a data race
noted in SURVEY §5.2). Here the whole library is compiled once into:

* a **regex registry**: every distinct regex string (primary, secondary, sequence event, plus
  the 4 built-in context regexes of ``ContextAnalysisService.java:27-34`` at ids 0..3) gets one
  id; its hits are computed once per request and shared by every pattern that references it;
* a **DFA pool** (byte DFAs of all regexes, concatenated) for the verify/scan kernels;
* **prefilter tables**: required literal factors of each regex, their leading 2/3/4-grams in a
  2-hash bloom filter (LDS-resident in the kernel) and an open-addressed hash table;
* **pattern tables** for the fused score kernel (confidence, severity multiplier, context rules,
  secondary / sequence descriptors, frequency key).

Every regular Java regex runs on the device: a byte DFA when its subset construction fits
``engine.dfa-max-states``, otherwise (bounded gaps ``X.{0,1000}Y``, repeated groups, MULTILINE
anchors, Unicode ``\b``) a bit-parallel Glushkov program over code points (``jregex.cpp``
bpg_program, ``csrc/kernels/bpg.h``). Only non-regular regexes (backreferences, lookaround,
possessive / atomic groups) use the host backtracker, as a side path run before the device
pipeline (``Engine.host_hits``); syntactically invalid regexes never match and are reported at load
(the reference would fail every request with a ``PatternSyntaxException`` -> HTTP 500).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..golden import CONTEXT_REGEXES, SEVERITY_MULTIPLIERS, java_blank, severity_key
from ..native import N
from ..utils.config import ScoringParams
from .nfa import build_group, fits_group, pack_groups
from .schema import Pattern, PatternSet, pattern_to_json

log = logging.getLogger("log_parser_amd.compiled")

KIND_DFA, KIND_NFA, KIND_FALLBACK, KIND_INVALID = 0, 1, 2, 3
RELAX = "(?#relax)"          # jregex: the automaton of the pattern's regular relaxation (a superset)
BLOOM_BITS = 18


def _minimize_literals(lits: List[bytes]) -> List[bytes]:
    """Drop literals that contain another literal of the same OR-set (redundant for a filter)."""
    s = sorted(set(lits), key=len)
    out: List[bytes] = []
    for x in s:
        if not any(y in x for y in out):
            out.append(x)
    return out


# Approximate byte frequencies (percent) of lower-cased log text: English letter frequencies
# scaled by the letter share, plus spaces, digits (timestamps, ids) and log punctuation. The
# prefilter gram of a literal is the window with the smallest estimated frequency. Digits are ~25%
# of log bytes (an ISO timestamp + a numeric id per line): at 1.2% each the model picked all-digit
# Teddy windows ("106" of the code "M106") that every id matches -- 680k false candidate
# positions per 12.5M-line step, half of k_pf_verify's work; at 3% it picks the code's letter.
_FREQ = {**{c: f * 0.55 for c, f in zip(b"etaoinshrdlcumwfgypbvkjxqz",
                                         (12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8, 2.4,
                                          2.4, 2.2, 2.0, 2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07))},
         **{c: 3.0 for c in b"0123456789"}, ord(" "): 14.0, ord("."): 1.5, ord(":"): 1.5, ord("-"): 1.2,
         ord("="): 0.6, ord("/"): 0.6, ord("_"): 0.5, ord("["): 0.4, ord("]"): 0.4, ord(","): 0.5,
         ord("("): 0.3, ord(")"): 0.3, ord("\t"): 0.5}


PF_STRIDE_MAX = 4      # largest prefilter sampling stride (1, 2 or 4); 1 disables sampling
PF_TEDDY = True        # short literals (3..6 bytes) on the byte-position (Teddy) tier
TEDDY_MIN, TEDDY_MAX = 3, 6
TEDDY_BUCKETS = 32
TEDDY_MAX_LITS = 2048  # beyond this the buckets saturate: extra short literals join the bloom tier
MIN_LITERAL = 3        # a regex whose required-literal set has a shorter member scans every line

# gram entries: gram_lits value = literal id | (window offset << LIT_OFF_SHIFT)
LIT_OFF_SHIFT = 22
MAX_GRAM_OFF = (1 << (31 - LIT_OFF_SHIFT)) - 1


def _window_cost(w: bytes) -> float:
    import math
    return sum(math.log2(_FREQ.get(c, 0.05) / 100.0) for c in w)


def _choose_grams(lits: List[bytes], stride: int = 1) -> List[List[Tuple[int, int, int]]]:
    """Per literal, the ``stride`` adjacent g-byte windows [(key, g, offset), ...] to index, rarest
    estimated text frequency first, with a mild penalty for windows already shared by other
    literals (each sharer costs a compare). With stride S in {2, 4} every occurrence of the literal
    has exactly one indexed window starting at a text position divisible by S, so the device
    prefilter tests every S-th position only (k_prefilter<GM, S>); callers pass stride S only when
    every literal has >= S + 3 bytes (S adjacent 4-byte windows)."""
    import math
    used: Dict[Tuple[int, int], int] = {}
    out = []
    for lit in lits:
        g = min(4, len(lit))
        best = None
        for i in range(min(len(lit) - g - stride + 1, MAX_GRAM_OFF - stride + 1) + 1):
            # expected verify work of the indexed windows = SUM over windows of text frequency x
            # bucket size (log domain: the worst window dominates; a rare partner does not excuse a
            # common or crowded one). Stride 1 keeps the milder sharing penalty it was tuned with.
            alpha = 0.5 if stride == 1 else 0.75
            cost = math.log2(sum(
                2.0 ** (_window_cost(lit[i + d:i + d + g])
                        + alpha * math.log2(1 + used.get((int.from_bytes(lit[i + d:i + d + g], "little"), g), 0)))
                for d in range(stride)))
            if best is None or (cost, i) < best:
                best = (cost, i)
        ents = []
        for d in range(stride):
            off = best[1] + d
            key = int.from_bytes(lit[off:off + g], "little")
            used[(key, g)] = used.get((key, g), 0) + 1
            ents.append((key, g, off))
        out.append(ents)
    return out


def _fingerprint(lit: bytes, off: int, g: int) -> Tuple[int, int]:
    """(fingerprint, mask) of one indexed window: the literal's (lower-cased) bytes in the 4 text
    positions before the window (low 32 bits) and the 4 after it (high 32 bits), where the literal
    has them. The device verify compares these 8 text bytes -- loaded once per gram hit -- against
    every literal of the bucket with ONE contiguous 16-byte load per literal, and walks the literal
    itself (3 dependent loads) only when they agree (k_pf_verify)."""
    fp = mask = 0
    for k in range(4):                     # text byte p - 4 + k  <->  literal byte off - 4 + k
        i = off - 4 + k
        if 0 <= i < len(lit):
            fp |= lit[i] << (8 * k)
            mask |= 0xFF << (8 * k)
    for k in range(4):                     # text byte p + g + k  <->  literal byte off + g + k
        i = off + g + k
        if i < len(lit):
            fp |= lit[i] << (32 + 8 * k)
            mask |= 0xFF << (32 + 8 * k)
    return fp, mask


def _fingerprints(entries: Sequence[int], lits: List[bytes], gs: Sequence[int]) -> np.ndarray:
    """uint64 [2 x len(entries)]: (fingerprint, mask) per bucket entry (literal id | offset << 22)
    whose indexed window is gs[j] bytes long."""
    out = np.zeros(2 * max(len(entries), 1), np.uint64)
    for j, e in enumerate(entries):
        lit = lits[e & ((1 << LIT_OFF_SHIFT) - 1)]
        fp, mask = _fingerprint(lit, e >> LIT_OFF_SHIFT, gs[j])
        out[2 * j], out[2 * j + 1] = np.uint64(fp), np.uint64(mask)
    return out


def _teddy_tables(lits: List[bytes], ids: List[int]):
    """Byte-position masks of the short-literal tier: (table uint32[256, 4] = M0 | M1 | M2 | 0 per
    byte value, bucket CSR offsets int32[B + 1], bucket entries = literal id | window offset << 22).
    Each literal indexes its rarest 3-byte window; literals are sorted by window and cut into
    contiguous buckets, so a bucket's members share leading bytes and its masks stay sparse."""
    tab = np.zeros((256, 4), np.uint32)
    if not lits:
        return tab, np.zeros(TEDDY_BUCKETS + 1, np.int32), np.zeros(1, np.int32)
    win = []
    for lit, i in zip(lits, ids):
        o = min(range(len(lit) - 2), key=lambda k: (_window_cost(lit[k:k + 3]), k))
        win.append((lit[o:o + 3], o, i))
    win.sort()
    B = min(TEDDY_BUCKETS, len(win))
    members: List[List[int]] = [[] for _ in range(TEDDY_BUCKETS)]
    for r, (w, o, i) in enumerate(win):
        b = r * B // len(win)
        for j in range(3):
            tab[w[j], j] |= np.uint32(1 << b)
        members[b].append(i | (o << LIT_OFF_SHIFT))
    off = np.zeros(TEDDY_BUCKETS + 1, np.int32)
    for b in range(TEDDY_BUCKETS):
        off[b + 1] = off[b] + len(members[b])
    ent = np.array([e for m in members for e in m] or [0], np.int32)
    return tab, off, ent


def _u32(x):
    return x & 0xFFFFFFFF


def bloom_hash(key, g):
    """Blocked bloom filter (csrc/kernels/lp_core.h): one 32-bit multiply per gram key."""
    return _u32((key ^ _u32(g * 0x9E3779B9)) * 0x85EBCA6B)


def bloom_word(key, g, bits):
    return bloom_hash(key, g) >> (32 - (bits - 5))


def bloom_bits2(key, g):
    p = bloom_hash(key, g)
    q = p ^ (p >> 15)
    return (1 << (q & 31)) | (1 << ((q >> 5) & 31)) | (1 << ((q >> 10) & 31))


def ht_hash(key, g):
    h = _u32(key * 0x9E3779B1) ^ _u32(g * 0x7FEB352D)
    h ^= h >> 15
    h = _u32(h * 0x2C1B3C6D)
    h ^= h >> 12
    return h


@dataclass
class RegexInfo:
    pattern: str
    kind: int
    error: str = ""
    literals: List[bytes] = field(default_factory=list)
    nstates: int = 0
    roles: set = field(default_factory=set)


class CompiledLibrary:
    def __init__(self, pattern_sets: List[PatternSet], params: ScoringParams, max_dfa_states: int = 2048,
                 nfa_engine: str = "bpg"):
        self.pattern_sets = pattern_sets
        self.params = params
        self.max_dfa_states = max_dfa_states
        # regexes whose DFA exceeds max_dfa_states: "bpg" = bit-parallel Glushkov programs run by the
        # DFA verify / scan kernels (models/bpg.py), "mfma" = the MFMA state-transition GEMM over
        # every line (<= 64 positions; A/B engine)
        if nfa_engine not in ("bpg", "mfma"):
            raise ValueError(f"engine.nfa-engine must be 'bpg' or 'mfma', not {nfa_engine!r}")
        self.nfa_engine = nfa_engine
        self.patterns: List[Pattern] = []
        self.pattern_set_index: List[int] = []
        for si, ps in enumerate(pattern_sets):
            for p in (ps.patterns or []):
                if p.primary_pattern is None or p.primary_pattern.regex is None:
                    log.error("pattern %r has no primary regex; skipped", p.id)
                    continue
                self.patterns.append(p)
                self.pattern_set_index.append(si)
        self.library_ids = [(ps.metadata.library_id if ps.metadata else None) for ps in pattern_sets]
        self._reg_ids: Dict[str, int] = {}
        self.regexes: List[RegexInfo] = []
        for rx in CONTEXT_REGEXES:
            self._reg(rx, "context")
        self._build_pattern_tables()
        self._compile_regexes()
        self._build_prefilter()
        self.pattern_json = [_json_bytes(pattern_to_json(p)) for p in self.patterns]
        self._device_cache: Dict[str, dict] = {}

    # ------------------------------------------------------------------ registry
    def _reg(self, rx: Optional[str], role: str) -> int:
        if rx is None:
            return -1
        i = self._reg_ids.get(rx)
        if i is None:
            i = len(self.regexes)
            self._reg_ids[rx] = i
            self.regexes.append(RegexInfo(pattern=rx, kind=-1))
        self.regexes[i].roles.add(role)
        return i

    def _build_pattern_tables(self):
        P = len(self.patterns)
        p = self.params
        self.conf = np.zeros(P, np.float64)
        self.sev = np.zeros(P, np.float64)
        self.severity = []
        # distinct severity strings (first appearance) and each pattern's index into them: the
        # summary kernel's severity histogram keys (severityDistribution, AnalysisService.java:197)
        self.sev_names: List[str] = []
        self.sev_index = np.zeros(P, np.int32)
        sev_of_name: Dict[str, int] = {}
        self.ctx_before = np.full(P, -1, np.int32)
        self.ctx_after = np.full(P, -1, np.int32)
        sec_off, sec_reg, sec_w, sec_weight = [0], [], [], []
        seq_off, seq_bonus, seq_ev_off, seq_ev_reg = [0], [], [0], []
        self.primary_reg = np.zeros(P, np.int32)
        self.freq_key = np.full(P, -1, np.int32)
        self.freq_ids: List[str] = []
        fid: Dict[str, int] = {}
        halo = 5
        for i, pat in enumerate(self.patterns):
            self.conf[i] = float(pat.primary_pattern.confidence)
            sk = severity_key(pat.severity)
            self.severity.append(sk)
            self.sev[i] = SEVERITY_MULTIPLIERS.get(sk, 1.0)
            if sk not in sev_of_name:
                sev_of_name[sk] = len(self.sev_names)
                self.sev_names.append(sk)
            self.sev_index[i] = sev_of_name[sk]
            ce = pat.context_extraction
            if ce is not None:
                self.ctx_before[i] = max(0, int(ce.lines_before))
                self.ctx_after[i] = max(0, int(ce.lines_after))
                halo = max(halo, self.ctx_before[i], self.ctx_after[i])
            self.primary_reg[i] = self._reg(pat.primary_pattern.regex, "primary")
            for s in (pat.secondary_patterns or []):
                sec_reg.append(self._reg(s.regex, "secondary"))
                w = min(p.max_window, int(s.proximity_window))
                sec_w.append(w)
                sec_weight.append(float(s.weight))
                halo = max(halo, w)
            sec_off.append(len(sec_reg))
            for q in (pat.sequence_patterns or []):
                seq_bonus.append(float(q.bonus_multiplier))
                for ev in (q.events or []):
                    seq_ev_reg.append(self._reg(ev.regex, "sequence"))
                seq_ev_off.append(len(seq_ev_reg))
            seq_off.append(len(seq_bonus))
            if not java_blank(pat.id):
                if pat.id not in fid:
                    fid[pat.id] = len(self.freq_ids)
                    self.freq_ids.append(pat.id)
                self.freq_key[i] = fid[pat.id]
        self.sec_off = np.array(sec_off, np.int32)
        self.sec_reg = np.array(sec_reg or [0], np.int32)
        self.sec_w = np.array(sec_w or [0], np.int32)
        self.sec_weight = np.array(sec_weight or [0.0], np.float64)
        self.seq_off = np.array(seq_off, np.int32)
        self.seq_bonus = np.array(seq_bonus or [0.0], np.float64)
        self.seq_ev_off = np.array(seq_ev_off, np.int32)
        self.seq_ev_reg = np.array(seq_ev_reg or [0], np.int32)
        self.n_seq_events = len(seq_ev_reg)
        self.halo = int(halo)
        # primary regex -> patterns (ascending pattern index = reference event order)
        R = len(self.regexes)
        cnt = np.zeros(R, np.int64)
        for r in self.primary_reg:
            cnt[r] += 1
        self.prim_off = np.zeros(R + 1, np.int64)
        np.cumsum(cnt, out=self.prim_off[1:])
        self.prim_pats = np.argsort(self.primary_reg, kind="stable").astype(np.int32)

    def bpg_program(self, r: int) -> np.ndarray:
        """The bit-parallel Glushkov program of regex ``r`` (a slice of ``bpg_pool``)."""
        if r not in self.bpg_regs:
            raise KeyError(f"regex {r} is not a BPG program")
        o = int(self.dfa_meta[r, 0])
        return self.bpg_pool[o:o + int(self.bpg_pool[o + 1] >> np.uint64(32))]

    def _compile_regexes(self):
        meta, bytemaps, trans, accs = [], [], [], []
        toff = aoff = 0
        bpgs: List[np.ndarray] = []
        boff = 0
        self.bpg_regs: List[int] = []
        self.bpg_scan_regs: List[int] = []
        self.scan_regs: List[int] = []
        self.host_regs: List[int] = []
        self.host_bt_ok: List[bool] = []
        self.host_lits: List[List[bytes]] = []        # backtracker regexes' required literals (host side path)
        # backtracker regexes whose REGULAR RELAXATION runs on the device (jregex Relaxer: a superset
        # language): its hits are only candidates, exported to the host backtracker (meta flag 4)
        self.host_dev: List[int] = []
        self.device_pattern: Dict[int, str] = {}
        nfa_members: List[Tuple[int, dict]] = []
        ctx_members: List[Tuple[int, dict]] = []
        self._ctx_ext = (0, 0)

        def add_dfa(d, flags=0):
            nonlocal toff, aoff
            meta.append([toff, d["nclasses"], aoff, (1 if d["anchored"] else 0) | flags])
            bytemaps.append(np.frombuffer(d["bytemap"], np.uint8))
            t = np.frombuffer(d["trans"], np.uint16)
            trans.append(t)
            a = np.frombuffer(d["acc"], np.uint8)
            accs.append(a)
            toff += t.size
            aoff += a.size

        def add_bpg(i, prog, flags=0):
            nonlocal boff
            meta.append([boff, 1, 0, 2 | flags])
            bytemaps.append(np.zeros(256, np.uint8))
            bpgs.append(prog)
            boff += prog.size
            self.bpg_regs.append(i)

        def dfa_literals(d):
            lits = _minimize_literals(list(d["literals"])) if d["has_literals"] else []
            if lits and min(len(x) for x in lits) < MIN_LITERAL:
                lits = []          # a 1-2-byte factor selects nothing: scan every line
            # anchored regexes (e.g. '^\\s*at\\s+...') die within a few bytes of every line:
            # scanning all lines beats a short, unselective literal.
            if d["anchored"] and lits and min(len(x) for x in lits) < 4:
                lits = []
            return lits

        for i, ri in enumerate(self.regexes):
            if i == 4:
                self._ctx_ext = (toff, aoff)     # the context DFAs' tables end here
            # the 4 context regexes are always DFAs: k_feat_cov walks their tables directly
            d = N.compile_regex(ri.pattern, max(self.max_dfa_states, 2048) if i < 4 else self.max_dfa_states, 4096)
            ri.kind = d["kind"]
            ri.error = d["error"]
            if i < 4:
                ctx_members.append((i, d))
            if ri.kind == KIND_DFA:
                ri.nstates = d["nstates"]
                add_dfa(d)
                lits = dfa_literals(d)
                if ri.roles == {"context"}:
                    # built-in context regexes are evaluated lazily, only on lines inside some
                    # event's context window (k_feat), never by the whole-log match stage
                    ri.literals = []
                    continue
                ri.literals = lits
                if not lits:
                    self.scan_regs.append(i)
            else:
                prog = None
                mfma_ok = ri.kind == KIND_NFA and d["npos"] > 0 and not d["cp_only"] and fits_group(d)
                if ri.kind == KIND_NFA and d["bpg"] and (self.nfa_engine == "bpg" or not mfma_ok):
                    prog = np.frombuffer(d["bpg"], np.uint64)
                if prog is not None:
                    # DFA blow-up (bounded gaps X.{0,1000}Y, repeated groups) or code-point contexts
                    # (MULTILINE anchors, Unicode \b): a bit-parallel Glushkov program over code
                    # points, dispatched by the verify / scan kernels next to the DFAs (meta bit 1)
                    ri.nstates = int(prog[0] & np.uint64(0xFF)) * 64
                    add_bpg(i, prog)
                    lits = _minimize_literals(list(d["literals"])) if d["has_literals"] else []
                    if lits and min(len(x) for x in lits) < MIN_LITERAL:
                        lits = []
                    ri.literals = lits if ri.roles != {"context"} else []
                    if not ri.literals:
                        self.bpg_scan_regs.append(i)      # every line, one lane per line (k_scan)
                    continue
                if ri.kind == KIND_FALLBACK and not mfma_ok and d.get("bt_ok") and ri.roles != {"context"}:
                    # non-regular (backref, lookaround, atomic, possessive): the host backtracker
                    # decides, but the device finds its candidate lines with the automaton of the
                    # regex's regular relaxation -- its literals through the prefilter, or, without
                    # one, its DFA in a literal-free scan group (meta flag 4: exported, never a hit)
                    dr = N.compile_regex(RELAX + ri.pattern, self.max_dfa_states, 4096)
                    rprog = np.frombuffer(dr["bpg"], np.uint64) if dr["kind"] == KIND_NFA and dr["bpg"] else None
                    if dr["kind"] == KIND_DFA or rprog is not None:
                        log.info("regex %r: host backtracker, device-fed by its relaxation", ri.pattern)
                        self.host_regs.append(i)
                        self.host_bt_ok.append(True)
                        lits = _minimize_literals(list(d["literals"])) if d["has_literals"] else []
                        self.host_lits.append(lits if lits and min(len(x) for x in lits) >= MIN_LITERAL else [])
                        self.host_dev.append(i)
                        self.device_pattern[i] = RELAX + ri.pattern
                        if rprog is not None:
                            add_bpg(i, rprog, 4)
                            lits = _minimize_literals(list(dr["literals"])) if dr["has_literals"] else []
                            ri.literals = lits if lits and min(len(x) for x in lits) >= MIN_LITERAL else []
                            if not ri.literals:
                                self.bpg_scan_regs.append(i)
                        else:
                            add_dfa(dr, 4)
                            ri.literals = dfa_literals(dr)
                            if not ri.literals:
                                self.scan_regs.append(i)
                        continue
                meta.append([0, 1, 0, 0])
                bytemaps.append(np.zeros(256, np.uint8))
                if ri.kind == KIND_INVALID:
                    log.error("invalid regex %r: %s (never matches)", ri.pattern, ri.error)
                elif mfma_ok:
                    # engine.nfa-engine=mfma: simulate the NFA with the MFMA state-transition kernel
                    nfa_members.append((i, d))
                else:
                    # no automaton even for its relaxation: the native backtracker on the host, as a
                    # side path before the device pipeline (Engine.host_hits) -- lines holding a
                    # required literal, or every line without one
                    log.info("regex %r runs on the host backtracker (%s)", ri.pattern, ri.error)
                    if not d.get("bt_ok"):
                        log.error("regex %r: no engine runs it (%s); it never matches", ri.pattern, ri.error)
                    self.host_regs.append(i)
                    self.host_bt_ok.append(bool(d.get("bt_ok")))
                    lits = _minimize_literals(list(d["literals"])) if d["has_literals"] else []
                    self.host_lits.append(lits if lits and min(len(x) for x in lits) >= MIN_LITERAL else [])
        # a dummy DFA for non-DFA regexes: state 2 -> DEAD on every byte (never read: not scanned)
        if not trans:
            trans.append(np.zeros(1, np.uint16))
            accs.append(np.zeros(1, np.uint8))
        # NFA groups for the MFMA kernel: the 4 context regexes first (one or two groups: the exact
        # UTF-8 '.' of the stack-frame regex costs ~10 positions), then DFA-blow-up regexes
        ctx_groups = pack_groups(ctx_members)
        groups = ctx_groups + pack_groups(nfa_members)
        tabs, ncls = zip(*[build_group(g) for g in groups])
        self.nfa_tables = np.concatenate(tabs)
        self.nfa_group_ncls = list(ncls)
        self.nfa_ctx_groups = list(range(len(ctx_groups)))
        self.nfa_ctx_ncls = max(ncls[:len(ctx_groups)])
        self.nfa_scan_groups = list(range(len(ctx_groups), len(groups)))
        self.nfa_regs = [rid for g in groups[len(ctx_groups):] for rid, _ in g]
        self._build_scan_passes()
        self.scan_regs_single = self.scan_regs_single + self.bpg_scan_regs
        self._build_host_matchers()
        self.bpg_pool = np.concatenate(bpgs) if bpgs else np.zeros(1, np.uint64)
        self.bpg_widths = 0                  # bit W: a program of W words exists (bpg.hip launches)
        for b in bpgs:        # (bit 31 stands for 32 words)
            self.bpg_widths |= 1 << min(31, int(b[0] & np.uint64(0xFF)))
        self.dfa_meta = np.array(meta, np.int32).reshape(-1, 4)
        self.dfa_bytemap = np.concatenate(bytemaps)
        self.dfa_trans = np.concatenate(trans)
        self.dfa_acc = np.concatenate(accs)

    def _build_host_matchers(self):
        """Backtracker regexes: native Java-semantics backtrackers (jregex BtRegex); a regex the
        backtracker rejects as well (e.g. \\N{name}) never matches (logged at load)."""
        self.host_bt = N.BtSet([self.regexes[r].pattern for r in self.host_regs]) if self.host_regs else None
        R = len(self.regexes)
        self.host_local = np.full(max(R, 1), -1, np.int32)      # global regex id -> index in host_bt
        for k, r in enumerate(self.host_regs):
            if self.host_bt is not None and self.host_bt.ok(k):
                self.host_local[r] = k
        # (local index, global id, required literals) of every runnable backtracker regex
        self.host_plan = [(int(self.host_local[r]), r, lits) for r, lits in zip(self.host_regs, self.host_lits)
                          if self.host_local[r] >= 0]
        # ... of those the device cannot feed (no automaton even for the relaxation): the host side
        # path scans the batch's bytes for them when the device feeds the others (side_path.hip)
        dev = set(self.host_dev)
        self.host_plan_undev = [x for x in self.host_plan if x[1] not in dev]
        self.host_dev_mask = np.zeros(max(R, 1), bool)
        self.host_dev_mask[self.host_dev] = True

    # multi-regex DFA scan groups (csrc/kernels/scan_multi.hip)
    SCAN_GROUP_REGS = 32            # members per multi-regex DFA (masks hold 64; one 46-member group
                                    # walked no faster than two groups in the bench step, profiles/r4_e)
    SCAN_GROUP_BYTES = 24 << 10     # LDS bytes of one group's uint16 transition rows
    SCAN_PASS_ROWS = 48 << 10       # LDS bytes of one pass's rows (+ 1 KiB bm4)
    SCAN_MAX_STATES = 4096

    @staticmethod
    def _row_stride(d) -> int:
        ncol = d["nclasses"] + 2                      # hold, '\n', classes
        return ncol if ncol % 2 else ncol + 1         # odd: rows start on spread-out banks

    def _dpat(self, r: int) -> str:
        """The pattern the device automata run for regex ``r`` (a backtracker regex: its relaxation)."""
        return self.device_pattern.get(r, self.regexes[r].pattern)

    def _build_scan_passes(self):
        """Literal-free regexes -> multi-regex DFA groups (greedy, in registry order: a regex joins
        the open group while the union DFA stays within the state / LDS budget) -> passes of up to
        4 groups whose tables fit in LDS together. A regex whose DFA alone does not fit stays on the
        one-regex-per-walk scan (``scan_regs_single``)."""
        groups: List[Tuple[List[int], dict]] = []
        single: List[int] = []
        cur: List[int] = []
        cur_d = None

        def fits(d):
            return (d is not None and 2 * (d["nclasses"] + 2) <= 255
                    and d["nstates"] * self._row_stride(d) * 2 <= self.SCAN_GROUP_BYTES)

        for r in self.scan_regs:
            if cur and len(cur) < self.SCAN_GROUP_REGS:
                d = N.compile_multi([self._dpat(x) for x in cur + [r]], self.SCAN_MAX_STATES)
                if fits(d):
                    cur.append(r)
                    cur_d = d
                    continue
            if cur:
                groups.append((cur, cur_d))
            d = N.compile_multi([self._dpat(r)], self.SCAN_MAX_STATES)
            if fits(d):
                cur, cur_d = [r], d
            else:
                cur, cur_d = [], None
                single.append(r)
        if cur:
            groups.append((cur, cur_d))
        self.scan_groups = groups
        self.scan_regs_single = single
        passes, cur_p, size = [], [], 0
        for regs, d in groups:
            gb = d["nstates"] * self._row_stride(d) * 2
            if cur_p and (len(cur_p) == 4 or size + gb > self.SCAN_PASS_ROWS):
                passes.append(cur_p)
                cur_p, size = [], 0
            cur_p.append((regs, d))
            size += gb
        if cur_p:
            passes.append(cur_p)
        self.scan_passes = [self._scan_blob(p) for p in passes]

    @classmethod
    def _scan_blob(cls, groups) -> dict:
        """One pass -> the blob of scan_multi.hip (uint32 words): [bm4 | u16 rows] staged in LDS,
        then the exact tables the rare path reads from global memory. States are renumbered so
        that the ones from which a member can accept come last (the hot loop's threshold test)."""
        BM_BYTES = 2048                                     # bm4 (512 entries) at LDS byte 0, rows after
        rows16, exact, emask, fins = [], [], [], []
        meta = {k: [0] * 4 for k in ("row_base", "stride", "thr", "init_row", "init_state", "ncol")}
        bm4 = np.zeros(256, np.uint32)
        base = BM_BYTES // 2                                # in uint16 entries
        for g, (regs, d) in enumerate(groups):
            ns, nc = d["nstates"], d["nclasses"]
            t = np.frombuffer(d["trans"], np.uint32).reshape(ns, nc)
            a = np.frombuffer(d["acc"], np.uint64).reshape(ns, nc)
            fin = np.frombuffer(d["fin"], np.uint64).reshape(ns, 2)
            accepting = (a != 0).any(axis=1) | (fin != 0).any(axis=1)
            order = np.concatenate([np.flatnonzero(~accepting), np.flatnonzero(accepting)])
            new_of = np.empty(ns, np.uint32)
            new_of[order] = np.arange(ns, dtype=np.uint32)
            ncol = nc + 2
            stride = cls._row_stride(d)
            init_new = int(new_of[1])
            # exact tables (state ids; accept masks indexed alike), rows in the new order
            ex = np.zeros((ns, ncol), np.uint32)
            ex[:, 0] = np.arange(ns, dtype=np.uint32)                         # hold
            ex[:, 1] = np.uint32(init_new)                                    # '\n': restart ...
            ex[:, 2:] = new_of[t[order]]
            em = np.zeros((ns, ncol), np.uint64)
            em[:, 1] = fin[order, 0]                                          # ... + EOL accepts
            em[:, 2:] = a[order]
            exact.append(ex.reshape(-1))
            emask.append(em.reshape(-1).view(np.uint32))              # u64 masks as (lo, hi) words
            fins.append(np.ascontiguousarray(fin[order]).reshape(-1).view(np.uint32))
            # LDS rows: byte offset of the next state's row
            rowb = (2 * (base + np.arange(ns, dtype=np.int64) * stride)).astype(np.int64)
            r16 = np.zeros((ns, stride), np.uint16)
            r16[:, :ncol] = rowb[ex].astype(np.uint16)
            rows16.append(r16.reshape(-1))
            meta["row_base"][g], meta["stride"][g] = 2 * base, stride
            meta["thr"][g] = int(2 * (base + int((~accepting).sum()) * stride))
            meta["init_row"][g], meta["init_state"][g], meta["ncol"][g] = int(rowb[init_new]), init_new, ncol
            base += ns * stride
            col2 = (np.frombuffer(d["bytemap"], np.uint8).astype(np.uint32) + np.uint32(2)) * np.uint32(2)
            col2[10] = 2                                                      # '\n': never inside a line
            bm4 |= col2 << np.uint32(8 * g)
        if 2 * base > 0xFFFF:
            raise ValueError("scan pass rows exceed the uint16 byte offset")
        r = np.concatenate(rows16)
        if r.size % 8:
            r = np.concatenate([r, np.zeros(8 - r.size % 8, np.uint16)])      # whole uint4 words
        parts = [bm4, np.zeros(256, np.uint32), r.view(np.uint32)]    # entries 256..511: hold
        off = 512 + r.size // 2
        lds_words = off
        gt_off, gm_off, fin_off = [0] * 4, [0] * 4, [0] * 4
        for g in range(len(groups)):
            gt_off[g] = off
            parts.append(exact[g])
            off += exact[g].size
        for g in range(len(groups)):
            gm_off[g] = off
            parts.append(emask[g])
            off += emask[g].size
        for g in range(len(groups)):
            fin_off[g] = off
            parts.append(fins[g])
            off += fins[g].size
        G = 64                                   # regex-id slots per group (scan_multi.hip scan_emit)
        rid = np.zeros(G * 4, np.uint32)
        for g, (regs, _) in enumerate(groups):
            rid[G * g:G * g + len(regs)] = regs
        rid_off = off
        parts.append(rid)
        off += rid.size
        # accept masks laid out like the LDS rows (u16 entry i of the LDS blob <-> u64 mask i): the
        # device's exact re-walk follows the LDS rows and loads each transition's mask with an
        # address known from the LDS chain -- 16 independent global loads per block instead of a
        # chain of 16 dependent exact-row loads
        am = np.zeros(2 * lds_words, np.uint64)
        for g, (regs, d) in enumerate(groups):
            ns, ncol, stride = d["nstates"], meta["ncol"][g], meta["stride"][g]
            b0 = meta["row_base"][g] // 2
            idx = b0 + np.arange(ns, dtype=np.int64)[:, None] * stride + np.arange(ncol, dtype=np.int64)[None, :]
            am[idx] = emask[g].view(np.uint64).reshape(ns, ncol)
        if off % 2:                              # 8-byte aligned u64 view on the device
            parts.append(np.zeros(1, np.uint32))
            off += 1
        am_off = off
        parts.append(am.view(np.uint32))
        blob = np.concatenate(parts)
        return dict(blob=blob, lds_words=lds_words, ngroups=len(groups), gt_off=tuple(gt_off),
                    fin_off=tuple(fin_off), gm_off=tuple(gm_off), bm_off=0, rid_off=rid_off, am_off=am_off,
                    regs=[x for regs, _ in groups for x in regs], **{k: tuple(v) for k, v in meta.items()})

    def _build_prefilter(self):
        """Two literal tiers, both tested by k_prefilter in one pass over the text:

        * long literals (>= 7 bytes): a blocked bloom filter of 4-byte windows in LDS, with
          stride-S sampling -- S adjacent windows per literal, every S-th text position tested;
        * short literals (3..6 bytes, ``PF_TEDDY``): a Teddy-style byte-position filter. Each
          literal picks its rarest 3-byte window and a bucket (<= 32); table entry c holds, for
          window offsets 0/1/2, the buckets whose window has byte c there, so a position is a
          candidate iff M0[b_p] & M1[b_p+1] & M2[b_p+2] != 0 -- one 16-byte LDS read per text
          byte instead of a hash per position, and one short literal no longer drags the whole
          library down to stride 1.

        Both tiers verify whole literals (k_pf_verify) before producing (regex, line) candidates."""
        lit_ids: Dict[bytes, int] = {}
        lit_regs: List[List[int]] = []
        for i, ri in enumerate(self.regexes):
            for lit in ri.literals:
                j = lit_ids.get(lit)
                if j is None:
                    j = len(lit_regs)
                    lit_ids[lit] = j
                    lit_regs.append([])
                lit_regs[j].append(i)
        lits = [None] * len(lit_ids)
        for k, v in lit_ids.items():
            lits[v] = k
        self.literals = lits
        lit_off = np.zeros(len(lits) + 1, np.int32)
        for i, l in enumerate(lits):
            lit_off[i + 1] = lit_off[i] + len(l)
        # 32 zero bytes of padding: the device literal compare reads 16-byte blocks past the end
        lit_bytes = np.frombuffer(b"".join(lits) + bytes(32), np.uint8).copy()
        lit_reg_off = np.zeros(len(lits) + 1, np.int32)
        for i, rr in enumerate(lit_regs):
            lit_reg_off[i + 1] = lit_reg_off[i] + len(rr)
        lit_reg = np.array([r for rr in lit_regs for r in rr] or [0], np.int32)
        # ---- tier split
        short = []
        if PF_TEDDY:
            short = [i for i, l in enumerate(lits) if TEDDY_MIN <= len(l) <= TEDDY_MAX and 0 not in l]
            short = short[:TEDDY_MAX_LITS]
        sset = set(short)
        long_ids = [i for i in range(len(lits)) if i not in sset]
        teddy, tb_off, tb_lits = _teddy_tables([lits[i] for i in short], short)
        # ---- bloom tier: stride-S sampling needs S adjacent 4-byte windows per literal (>= S + 3 bytes)
        grams: Dict[Tuple[int, int], List[int]] = {}
        gmask = 0
        stride = 1
        if long_ids and len(lits) < (1 << LIT_OFF_SHIFT):
            shortest = min(len(lits[i]) for i in long_ids)
            for s_ in (4, 2):
                if PF_STRIDE_MAX >= s_ and shortest >= s_ + 3:
                    stride = s_
                    break
        for i, ents in zip(long_ids, _choose_grams([lits[i] for i in long_ids], stride)):
            for key, g, off in ents:
                grams.setdefault((key, g), []).append(i | (off << LIT_OFF_SHIFT))
                gmask |= 1 << g
        bits = BLOOM_BITS
        bloom = np.zeros((1 << bits) // 32, np.uint32)
        for key, g in grams:
            bloom[bloom_word(key, g, bits)] |= np.uint32(bloom_bits2(key, g))
        H = 16
        while H < 2 * max(1, len(grams)):
            H *= 2
        ht_key = np.full(H, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
        ht_val = np.zeros(H, np.int32)
        ht_cnt = np.zeros(H, np.int32)
        gram_lits: List[int] = []
        gram_g: List[int] = []
        for (key, g), ids in grams.items():
            h = ht_hash(key, g) & (H - 1)
            while ht_key[h] != np.uint64(0xFFFFFFFFFFFFFFFF):
                h = (h + 1) & (H - 1)
            ht_key[h] = np.uint64(key | (g << 32))
            ht_val[h] = len(gram_lits)
            ht_cnt[h] = len(ids)
            gram_lits.extend(ids)
            gram_g.extend([g] * len(ids))
        gram_fp = _fingerprints(gram_lits, lits, gram_g)
        ntb = int(tb_off[-1])
        tb_fp = _fingerprints([int(x) for x in tb_lits[:ntb]], lits, [3] * ntb)
        self.pf = dict(gram_g=np.array(gram_g or [4], np.int32), bloom=bloom, bits=bits, ht_key=ht_key, ht_val=ht_val, ht_cnt=ht_cnt, ht_mask=H - 1,
                       gram_fp=gram_fp, tb_fp=tb_fp,
                       gram_lits=np.array(gram_lits or [0], np.int32), lit_off=lit_off, lit_bytes=lit_bytes,
                       lit_reg_off=lit_reg_off, lit_reg=lit_reg, gmask=gmask, stride=stride,
                       teddy=teddy, tb_off=tb_off, tb_lits=tb_lits, teddy_lits=len(short))

    # ------------------------------------------------------------------ device tables
    def device_tables(self, device: torch.device) -> dict:
        key = str(device)
        t = self._device_cache.get(key)
        if t is not None:
            return t

        def T(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(device)

        t = {}
        pf = self.pf
        t["pf_arrays"] = [T(pf["bloom"]), T(pf["ht_key"].view(np.int64)), T(pf["ht_val"]), T(pf["ht_cnt"]),
                          T(pf["gram_lits"]), T(pf["lit_off"]), T(pf["lit_bytes"]), T(pf["lit_reg_off"]),
                          T(pf["lit_reg"]), T(pf["teddy"]), T(pf["tb_off"]), T(pf["tb_lits"]),
                          T(pf["gram_fp"].view(np.int64)), T(pf["tb_fp"].view(np.int64))]
        a = t["pf_arrays"]
        t["pf"] = (a[0].data_ptr(), pf["bits"], a[1].data_ptr(), a[2].data_ptr(), a[3].data_ptr(), pf["ht_mask"],
                   a[4].data_ptr(), a[5].data_ptr(), a[6].data_ptr(), a[7].data_ptr(), a[8].data_ptr(), pf["gmask"],
                   pf["stride"], a[9].data_ptr(), a[10].data_ptr(), a[11].data_ptr(), 1 if pf["teddy_lits"] else 0,
                   a[12].data_ptr(), a[13].data_ptr())
        t["dfa_arrays"] = [T(self.dfa_meta), T(self.dfa_bytemap), T(self.dfa_trans.view(np.int16)), T(self.dfa_acc),
                           T(self.bpg_pool.view(np.int64))]
        d = t["dfa_arrays"]
        t["dfa"] = (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), d[4].data_ptr(),
                    self.bpg_widths, int(self.bpg_pool.size))
        t["scan_regs"] = T(np.array(self.scan_regs_single, np.int32))
        t["scan_blobs"] = [T(p["blob"]) for p in self.scan_passes]
        t["scan_passes"] = [(b.data_ptr(), p["lds_words"], p["ngroups"], p["row_base"], p["stride"], p["thr"],
                             p["init_row"], p["init_state"], p["ncol"], p["gt_off"], p["fin_off"], p["bm_off"],
                             p["rid_off"], p["am_off"], p["gm_off"]) for b, p in zip(t["scan_blobs"], self.scan_passes)]
        t["conf"], t["sev"] = T(self.conf), T(self.sev)
        t["sev_index"] = T(self.sev_index)
        t["ctx_before"], t["ctx_after"] = T(self.ctx_before), T(self.ctx_after)
        t["sec_off"], t["sec_reg"], t["sec_w"], t["sec_weight"] = T(self.sec_off), T(self.sec_reg), T(self.sec_w), T(self.sec_weight)
        t["seq_off"], t["seq_bonus"], t["seq_ev_off"], t["seq_ev_reg"] = T(self.seq_off), T(self.seq_bonus), T(self.seq_ev_off), T(self.seq_ev_reg)
        slot_seq = np.zeros(max(self.n_seq_events, 1), np.int32)
        for q in range(len(self.seq_off) and (self.seq_ev_off.size - 1)):
            slot_seq[self.seq_ev_off[q]:self.seq_ev_off[q + 1]] = q
        t["slot_seq"] = T(slot_seq)
        t["prim_off"], t["prim_pats"] = T(self.prim_off), T(self.prim_pats)
        t["prim_cnt"] = T(np.diff(self.prim_off))
        t["freq_key"] = T(self.freq_key)
        t["is_primary"] = T(np.diff(self.prim_off) > 0)
        t["host_dev"] = bool(self.host_dev)          # backtracker regexes fed by their relaxed automata
        t["nfa_tables"] = T(self.nfa_tables.view(np.int64))
        t["nfa_ctx_list"] = T(np.array(self.nfa_ctx_groups, np.int32))
        t["nfa_scan_lists"] = {k: T(np.array([g for g in self.nfa_scan_groups if self.nfa_group_ncls[g] == k], np.int32))
                               for k in (1, 2, 3)}
        self._device_cache[key] = t
        return t

    @property
    def ctx_dfa_extent(self) -> Tuple[int, int]:
        """(trans, acc) entries spanned by the 4 context DFAs (pool entries 0..3, offset 0): the
        context-feature kernel stages exactly this prefix of the pool in LDS. (Recorded while the
        pool is laid out: entry 4 may be a BPG program or a host regex, whose meta holds no DFA
        offsets.)"""
        if len(self.regexes) > 4:
            return self._ctx_ext
        return int(self.dfa_trans.size), int(self.dfa_acc.size)

    @property
    def n_regexes(self) -> int:
        return len(self.regexes)

    def summary(self) -> dict:
        kinds = [r.kind for r in self.regexes]
        return {
            "patterns": len(self.patterns), "pattern_sets": len(self.pattern_sets), "regexes": len(self.regexes),
            "dfa": kinds.count(KIND_DFA), "host_fallback": len(self.host_regs), "host_device_fed": len(self.host_dev),
            "host_backtracker": int((self.host_local >= 0).sum()) if self.host_regs else 0,
            "invalid": kinds.count(KIND_INVALID), "scan_all": len(self.scan_regs), "literals": len(self.literals),
            "teddy_literals": int(self.pf["teddy_lits"]), "prefilter_stride": int(self.pf["stride"]),
            "scan_groups": len(self.scan_groups), "scan_passes": len(self.scan_passes),
            "nfa_mfma": len(self.nfa_regs), "nfa_groups": len(self.nfa_scan_groups),
            "nfa_bpg": len(self.bpg_regs), "nfa_bpg_scan_all": len(self.bpg_scan_regs),
            "halo": self.halo,
        }


def _json_bytes(obj) -> bytes:
    import json
    return json.dumps(obj, ensure_ascii=False, separators=(",", ":"), allow_nan=True).encode("utf-8")
