"""Torch-facing wrappers of the native kernels.

Each op takes torch tensors; CUDA (HIP) tensors run the gfx950 kernel on the current stream,
CPU tensors run the host twin compiled from the same source (``csrc/kernels/lp_core.h``).
There is no silent fallback: a CUDA tensor with a missing extension raises.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..native import N

# pad every device text buffer so vector loads past the end stay in bounds
TEXT_PAD = 64
NL_TILE = 16384


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def padded_len(nbytes: int) -> int:
    return ((max(nbytes, 1) + NL_TILE - 1) // NL_TILE) * NL_TILE + TEXT_PAD


def newline_positions(text: torch.Tensor, nbytes: int) -> torch.Tensor:
    """Positions of every '\\n' in text[0:nbytes] (int64, ascending; host twin)."""
    c = N.nl_positions_host(text.data_ptr(), nbytes, 0)
    pos = torch.empty(c, dtype=torch.int64)
    N.nl_positions_host(text.data_ptr(), nbytes, pos.data_ptr())
    return pos


class _LineIndexWs:
    """Per (device, stream) scratch of the line index: tile counts + offsets, "\\r\\n" flags and
    each tile's first line end (k_line_fix), the per-tile newline bitmasks (256 words = 2 KiB per
    16 KiB tile), then the scan scratch. Grow-only; stream order makes reuse safe."""
    SCAN_TMP = 1 << 20           # bytes of scan scratch in the workspace layout (csrc/bind.cpp passes the same)
    WORDS_PER_TILE = 4 + 256     # int64 words per tile (csrc/kernels/line_index.hip line_index_dev)
    _all: dict = {}

    @classmethod
    def get(cls, text: torch.Tensor, ntiles: int) -> Tuple[int, int]:
        key = (text.device, _s(text))
        buf = cls._all.get(key)
        w = cls.WORDS_PER_TILE
        if buf is None or buf.numel() < w * ntiles + cls.SCAN_TMP // 8:
            cap = max(ntiles * 5 // 4, 1024)
            buf = cls._all[key] = torch.empty(w * cap + cls.SCAN_TMP // 8, dtype=torch.int64, device=text.device)
        return buf.data_ptr(), (buf.numel() - cls.SCAN_TMP // 8) // w


# lines per byte seen so far (grows only): capacity of the line index outputs, so the one-pass
# kernel rarely needs a second pass; a text with more lines than that re-runs with the exact count
_LINES_PER_BYTE = [1.0 / 48]

import threading as _threading

_count_read = _threading.local()     # per thread: the pinned 24-byte count buffer + its event


def _count_read_slot(device: torch.device):
    """(pinned int64[3], event) reused by this thread's line-index count reads on ``device`` (a
    fresh pinned allocation and event per call cost host time on config 2's critical path; the
    buffer is read before the call returns, so one per thread and device suffices)."""
    slots = getattr(_count_read, "slots", None)
    if slots is None:
        slots = _count_read.slots = {}
    slot = slots.get(device.index)
    if slot is None:
        slot = slots[device.index] = (torch.empty(3, dtype=torch.int64, pin_memory=True), torch.cuda.Event())
    return slot
LINE_BLK_SHIFT = 12


def _line_index_dev(text: torch.Tensor, nbytes: int, trim: bool, before_read=None, fused=None,
                    early_first: bool = False):
    """k_nl_count, k_tile_scan, k_nl_lines, k_line_fix (+ k_line_trim): (starts, lens, n_newlines,
    last_newline, kept, blk) with ONE host read; blk = the coarse 4 KiB block -> line index.
    ``before_read()`` runs once, after the launches and before that read: work it queues (the
    literal prefilter, which needs no line index) runs on the GPU while the host waits.
    ``fused(nlp)`` instead launches the literal prefilter FIRST with the line index's first pass
    folded into its read of the text (nlp = the pass-1 outputs, zeroed): k_nl_count does not run.
    ``early_first``: before_read() queues its work on ANOTHER stream -- it then runs before the
    count copy is even set up, so that work is launched as soon as the line index is."""
    dev = text.device
    nt = N.line_index_tiles(nbytes)
    cap = int(nbytes * _LINES_PER_BYTE[0] * 1.25) + 1024
    blk = torch.empty((max(nbytes, 1) >> LINE_BLK_SHIFT) + 2, dtype=torch.int32, device=dev)
    counted = False
    while True:
        cap = min(cap, nbytes + 1)
        starts = torch.empty(cap, dtype=torch.int64, device=dev)
        lens = torch.empty(cap, dtype=torch.int32, device=dev)
        info = torch.empty(3, dtype=torch.int64, device=dev)
        wp, wcap = _LineIndexWs.get(text, nt)
        if fused is not None:
            fused(N.line_index_pass1(wp, wcap, nbytes, _s(text)))
            fused = None
            counted = True            # a re-run (more lines than the capacity) reuses pass 1's outputs
        N.line_index_dev(text.data_ptr(), nbytes, wp, wcap, starts.data_ptr(), lens.data_ptr(), cap, info.data_ptr(),
                         trim, blk.data_ptr(), blk.numel(), _s(text), counted)
        if before_read is not None:
            # the counts travel to pinned memory behind the line index only; the host then waits
            # for that copy, not for the work before_read() queued after it
            if early_first:
                before_read()
            hinfo, done = _count_read_slot(dev)
            hinfo.copy_(info, non_blocking=True)
            done.record()
            if not early_first:
                before_read()
            before_read = None
            done.synchronize()
            n_nl, last, kept = hinfo.tolist()
        else:
            n_nl, last, kept = info.tolist()
        if n_nl + 1 <= cap:
            _LINES_PER_BYTE[0] = max(_LINES_PER_BYTE[0], (n_nl + 1) / max(nbytes, 1))
            return starts, lens, n_nl, last, kept, blk
        cap = n_nl + 1


def _with_blk(ls: torch.Tensor, blk: torch.Tensor, nbytes: int) -> torch.Tensor:
    """Attach the coarse block index to the line-start tensor the caller gets (reused by
    ``line_block_index`` for the same object; any other tensor recomputes it)."""
    ls._lp_blk = (blk, nbytes)
    return ls


def split_lines(text: torch.Tensor, nbytes: int, before_read=None, fused=None,
                early_first: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Java ``logs.split("\\\\r?\\\\n")`` line index (AnalysisService.java:53).

    Returns (line_start int64[L], line_len int32[L]); trailing empty lines removed; input
    without any newline is one line (possibly empty). GPU: one read of the text + its newline bitmask, five small
    launches, one 24-byte host read (csrc/kernels/line_index.hip).
    """
    dev = text.device
    if text.is_cuda:
        if nbytes == 0:
            return torch.zeros(1, dtype=torch.int64, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)
        starts, lens, _, _, L, blk = _line_index_dev(text, nbytes, trim=True, before_read=before_read, fused=fused,
                                                     early_first=early_first)
        return _with_blk(starts[:L], blk, nbytes), lens[:L]
    nl = newline_positions(text, nbytes)
    if nl.numel() == 0:
        return (torch.zeros(1, dtype=torch.int64, device=dev),
                torch.full((1,), nbytes, dtype=torch.int32, device=dev))
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    starts = torch.cat([zero, nl + 1])
    ends = torch.cat([nl, torch.full((1,), nbytes, dtype=torch.int64, device=dev)])
    prev = text[(nl - 1).clamp(min=0)]
    cr = (nl > starts[:-1]) & (prev == 13)
    ends[:-1] -= cr.to(torch.int64)
    lens = ends - starts
    nz = torch.nonzero(lens > 0)
    L = int(nz[-1].item()) + 1 if nz.numel() else 0
    return starts[:L].contiguous(), lens[:L].to(torch.int32).contiguous()


def split_chunk_lines(text: torch.Tensor, nbytes: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Line index of a chunk made of complete lines (streaming): no trailing-empty trimming; a
    final '\\n' terminates the last line instead of opening an empty one."""
    dev = text.device
    if text.is_cuda and nbytes > 0:
        starts, lens, n_nl, last, _, blk = _line_index_dev(text, nbytes, trim=False)
        L = n_nl + 1 - (1 if n_nl and last == nbytes - 1 else 0)
        return _with_blk(starts[:L], blk, nbytes), lens[:L]
    nl = newline_positions(text.cpu(), nbytes).to(dev)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    starts = torch.cat([zero, nl + 1])
    ends = torch.cat([nl, torch.full((1,), nbytes, dtype=torch.int64, device=dev)])
    if nl.numel():
        prev = text[(nl - 1).clamp(min=0)]
        cr = (nl > starts[:-1]) & (prev == 13)
        ends[:-1] -= cr.to(torch.int64)
    L = starts.numel()
    if nl.numel() and int(nl[-1].item()) == nbytes - 1:
        L -= 1
    return starts[:L].contiguous(), (ends - starts)[:L].to(torch.int32).contiguous()




def line_block_index(line_start: torch.Tensor, nbytes: int) -> torch.Tensor:
    """blk[b] = line containing byte b << 12 (int32), for O(log lines-per-4KiB) line lookups
    (already built by the GPU line index for the tensors ``split_lines`` returns)."""
    cached = getattr(line_start, "_lp_blk", None)
    if cached is not None and cached[1] == nbytes:
        return cached[0]
    nblk = (max(nbytes, 1) >> LINE_BLK_SHIFT) + 2
    blk = torch.empty(nblk, dtype=torch.int32, device=line_start.device)
    N.blk_index(line_start.data_ptr(), line_start.numel(), nblk, blk.data_ptr(), _s(line_start), line_start.is_cuda)
    return blk


def prefilter(text, nbytes, pf_tuple, line_start, cap: int, grid: int = 2048) -> torch.Tensor:
    """Literal prefilter -> (regex << 32 | line) candidates (unverified, may repeat).

    GPU: k_prefilter streams the text and stages bloom gram hits (position, gram length);
    k_pf_verify then checks whole literals, one lane per hit, reading the gram-hit count on the
    device (grid-stride) -- both counts come back in ONE host read.
    """
    nlines = line_start.numel()
    if text.is_cuda:
        dev = text.device
        gcap = cap
        blk = line_block_index(line_start, nbytes)
        while True:
            gh = torch.empty(max(gcap, 1), dtype=torch.int64, device=dev)
            cand = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
            cnt = torch.zeros(2, dtype=torch.int64, device=dev)        # [gram hits, candidates]
            N.prefilter_dev(text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(), nlines, gh.data_ptr(), gcap,
                            cnt.data_ptr(), grid, _s(text))
            N.pf_verify_dev(gh.data_ptr(), gcap, text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(), nlines,
                            blk.data_ptr(), cand.data_ptr(), cap, cnt.data_ptr() + 8, _s(text), cnt.data_ptr(),
                            max(16, min(8192, nbytes >> 13)))   # grid-stride over the device count
            c = cnt.cpu()
            g, k = int(c[0]), int(c[1])
            if g <= gcap and k <= cap:
                return cand[:k]
            gcap, cap = max(gcap, g), max(cap, k)
    while True:
        cand = torch.empty(max(cap, 1), dtype=torch.int64)
        c = N.prefilter_host(text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(), nlines, cand.data_ptr(), cap)
        if c <= cap:
            return cand[:c]
        cap = c


def scan(text, line_start, line_len, regs: torch.Tensor, dfa_tuple, cap: int) -> torch.Tensor:
    nlines = line_start.numel()
    if regs.numel() == 0 or nlines == 0:
        return torch.empty(0, dtype=torch.int64, device=text.device)
    if text.is_cuda:
        while True:
            out = torch.empty(max(cap, 1), dtype=torch.int64, device=text.device)
            cnt = torch.zeros(1, dtype=torch.int64, device=text.device)
            N.scan_dev(text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(), nlines, regs.data_ptr(),
                       regs.numel(), dfa_tuple, out.data_ptr(), cap, cnt.data_ptr(), _s(text))
            c = int(cnt.item())
            if c <= cap:
                return out[:c]
            cap = c
    while True:
        out = torch.empty(max(cap, 1), dtype=torch.int64)
        c = N.scan_host(text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(), nlines, regs.data_ptr(),
                        regs.numel(), dfa_tuple, out.data_ptr(), cap)
        if c <= cap:
            return out[:c]
        cap = c


def scan_multi(text, nbytes: int, line_start, line_len, pass_tuple, cap: int, grid: int = 1024) -> torch.Tensor:
    """Literal-free regexes of one scan pass (<= 4 multi-regex DFA groups) over every line ->
    (regex << 32 | line) hits, already verified."""
    nlines = line_start.numel()
    if nlines == 0:
        return torch.empty(0, dtype=torch.int64, device=text.device)
    while True:
        out = torch.empty(max(cap, 1), dtype=torch.int64, device=text.device)
        if text.is_cuda:
            cnt = torch.zeros(1, dtype=torch.int64, device=text.device)
            N.scan_multi(text.data_ptr(), nbytes, line_start.data_ptr(), line_len.data_ptr(), nlines, pass_tuple,
                         out.data_ptr(), cap, cnt.data_ptr(), grid, _s(text), True)
            c = int(cnt.item())
        else:
            c = N.scan_multi(text.data_ptr(), nbytes, line_start.data_ptr(), line_len.data_ptr(), nlines, pass_tuple,
                             out.data_ptr(), cap, 0, 0, 0, False)
        if c <= cap:
            return out[:c]
        cap = c


def nfa_features(groups: torch.Tensor, lines: torch.Tensor, L: int, text, line_start, line_len,
                 group_list: torch.Tensor, ncls: int) -> torch.Tensor:
    """Context features via the MFMA NFA kernel (``group_list`` = the groups of the 4 context
    regexes, one launch each: a group ORs its members' bits into the line's byte): uint8 bits per line."""
    feat = torch.zeros(max(L, 1), dtype=torch.uint8, device=text.device)
    if lines.numel():
        for k in range(group_list.numel()):
            N.nfa(groups.data_ptr(), group_list[k:k + 1].data_ptr(), 1, ncls, lines.data_ptr(), lines.numel(),
                  text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(), feat.data_ptr(), 0, 0, 0, _s(text),
                  text.is_cuda)
    return feat


def nfa_scan(groups: torch.Tensor, group_list: torch.Tensor, ncls: int, text, line_start, line_len,
             cap: int) -> torch.Tensor:
    """All lines x NFA groups -> (regex << 32 | line) hits (MFMA kernel on GPU, bitset twin on CPU)."""
    nl = line_start.numel()
    if group_list.numel() == 0 or nl == 0:
        return torch.empty(0, dtype=torch.int64, device=text.device)
    while True:
        out = torch.empty(max(cap, 1), dtype=torch.int64, device=text.device)
        if text.is_cuda:
            cnt = torch.zeros(1, dtype=torch.int64, device=text.device)
            N.nfa(groups.data_ptr(), group_list.data_ptr(), group_list.numel(), ncls, 0, nl, text.data_ptr(),
                  line_start.data_ptr(), line_len.data_ptr(), 0, out.data_ptr(), cap, cnt.data_ptr(), _s(text), True)
            c = int(cnt.item())
        else:
            c = N.nfa(groups.data_ptr(), group_list.data_ptr(), group_list.numel(), ncls, 0, nl, text.data_ptr(),
                      line_start.data_ptr(), line_len.data_ptr(), 0, out.data_ptr(), cap, 0, 0, False)
        if c <= cap:
            return out[:c]
        cap = c


# ---------------------------------------------------------------------------------------------
# post-match pipeline (csrc/kernels/lp_post.hip): hit CSR, events, frequency ranks, features

class Uploader:
    """Several small host arrays -> device with ONE async H2D copy through a grow-only pinned
    buffer (line index, segment table, frequency carry of a request batch). CPU: zero-copy views.
    Reusing the pinned buffer is safe: every batch ends with a blocking read of its results,
    which orders after this copy on the same stream."""

    def __init__(self, device: torch.device):
        self.device = device
        self.pinned: Optional[torch.Tensor] = None

    def __call__(self, arrays):
        import numpy as np
        arrays = [np.ascontiguousarray(a) for a in arrays]
        if self.device.type != "cuda":
            return [torch.from_numpy(a) for a in arrays]
        offs, o = [], 0
        for a in arrays:
            offs.append(o)
            o += (a.nbytes + 255) // 256 * 256
        o = max(o, 256)
        if self.pinned is None or self.pinned.numel() < o:
            self.pinned = torch.empty(max(o * 5 // 4, 1 << 16), dtype=torch.uint8, pin_memory=True)
        hv = self.pinned.numpy()
        for a, off in zip(arrays, offs):
            hv[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
        dev = torch.empty(o, dtype=torch.uint8, device=self.device)
        dev.copy_(self.pinned[:o], non_blocking=True)
        return [dev[off:off + a.nbytes].view(_TORCH_DTYPE[a.dtype.str]) for a, off in zip(arrays, offs)]


_TORCH_DTYPE = {"<i8": torch.int64, "<i4": torch.int32, "<u1": torch.uint8, "<f8": torch.float64, "|u1": torch.uint8,
                "|b1": torch.bool}


class Workspace:
    """Grow-only device scratch buffer for the post-match kernels' temporaries (rocPRIM temp
    storage, sort ping-pong buffers, window difference array). One per engine; stream-ordered
    reuse is safe because every batch ends with a host read of its results."""

    def __init__(self, device: torch.device):
        self.device = device
        self.buf: Optional[torch.Tensor] = None

    def get(self, nbytes: int) -> Tuple[int, int]:
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(int(nbytes * 5 // 4), 1 << 20), dtype=torch.uint8, device=self.device)
        return self.buf.data_ptr(), self.buf.numel()

    def ptr(self) -> Tuple[int, int]:
        return (0, 0) if self.buf is None else (self.buf.data_ptr(), self.buf.numel())


def _run_ws(call, ws: Optional[Workspace]):
    """Device calls report the workspace they need and run only when it suffices."""
    p, n = ws.ptr()
    need = call(p, n)
    if need > n:
        p, n = ws.get(need)
        call(p, n)


def ev_tables(tabs: dict, segs, nkeys: int, npat: int) -> tuple:
    return (tabs["prim_off"].data_ptr(), tabs["prim_pats"].data_ptr(), tabs["freq_key"].data_ptr(),
            tabs["ctx_before"].data_ptr(), tabs["ctx_after"].data_ptr(), segs.lo.data_ptr(), segs.hi.data_ptr(),
            segs.own_lo.data_ptr(), segs.own_hi.data_ptr(), segs.lo.numel(), nkeys, N.bits_for(max(npat, 1)))


def post_hits(cand: torch.Tensor, pre_from: int, L: int, R: int, text, line_start, line_len, dfa_tuple,
              evt: tuple, ws: Optional[Workspace]):
    """Candidates -> (hits, hit_line, hit_off, ev_cnt, ev_end, n_hits, n_events).

    ``cand[:pre_from]`` are prefilter candidates still to DFA-verify, ``cand[pre_from:]`` hits of
    engines that verified already (scan / MFMA NFA / host fallback). Duplicates are allowed.
    Output hits are sorted unique (regex << 32 | line); one 16-byte host read for the counts."""
    dev = cand.device
    n = cand.numel()
    m = max(n, 1)
    hits = torch.empty(m, dtype=torch.int64, device=dev)
    hit_line = torch.empty(m, dtype=torch.int32, device=dev)
    hit_off = torch.empty(R + 1, dtype=torch.int64, device=dev)
    ev_cnt = torch.empty(m, dtype=torch.int64, device=dev)
    ev_end = torch.empty(m, dtype=torch.int64, device=dev)
    counters = torch.empty(2, dtype=torch.int64, device=dev)      # written by the pipeline
    lbits, rbits = N.bits_for(max(L, 1)), N.bits_for(max(R, 1))

    def call(wp, wn):
        return N.post_hits(cand.data_ptr(), n, pre_from, lbits, rbits, R, text.data_ptr(), line_start.data_ptr(),
                           line_len.data_ptr(), dfa_tuple, evt, hits.data_ptr(), hit_line.data_ptr(),
                           hit_off.data_ptr(), ev_cnt.data_ptr(), ev_end.data_ptr(), counters.data_ptr(), wp, wn,
                           _s(cand), cand.is_cuda, 0, 0)

    if cand.is_cuda:
        _run_ws(call, ws)
        c = counters.cpu()
    else:
        call(0, 0)
        c = counters
    nh, ne = int(c[0]), int(c[1])
    return hits[:nh], hit_line, hit_off, ev_cnt, ev_end, nh, ne


class MatchArena:
    """Fixed-capacity device buffers of every matcher of one batch + their append counters
    (GPU): gram hits (k_prefilter), prefilter candidates (k_pf_verify), verified hits of the
    self-verifying engines (scan passes, single-DFA scan, MFMA NFA). Nothing is read back until
    the hit CSR is built, so matching + verify + CSR + event count cost ONE host read
    (``match_and_hits``); capacities follow the largest per-line rates seen so far, and a batch
    that overflows one re-runs with its exact counts."""

    def __init__(self):
        # starting rates per line (an underestimate costs one re-run of the matchers; an
        # overestimate costs post-match work on every batch, which covers the capacity); "ev":
        # events, only for steps that defer the count read (``match_and_hits(defer=True)``)
        self.rate = {"gram": 0.08, "cand": 0.03, "ver": 0.01, "ev": 0.01}
        self.last: dict = {}            # counts of the latest batch (diagnostics)

    def caps(self, L: int) -> dict:
        return {k: int(L * r * 1.25) + 512 for k, r in self.rate.items()}

    @staticmethod
    def overflow(counts: list, caps: dict) -> bool:
        """counts = [gram, cand, ver, nh, ne] of a deferred step vs its capacities."""
        g, k, v, _, ne = counts
        return g > caps["gram"] or k > caps["cand"] or v > caps["ver"] or ne > caps["ev"]

    def learn_deferred(self, L: int, counts: list) -> None:
        g, k, v, nh, ne = counts
        self.last = {"lines": L, "gram_hits": g, "prefilter_candidates": k, "scan_hits": v, "hits": nh, "events": ne}
        self.learn(L, {"gram": g, "cand": k, "ver": v, "ev": ne}, overflow=False)

    def learn(self, L: int, counts: dict, overflow: bool) -> None:
        """Overflow: the exact rates. Otherwise decay toward what batches need (the hit sort
        covers the whole capacity, so slack costs sort time)."""
        for k, c in counts.items():
            r = c / max(L, 1)
            self.rate[k] = max(r, self.rate[k] if overflow else self.rate[k] * 0.5, 1e-4)


def _pf_events(stream: "torch.cuda.Stream"):
    """(fork, done) events of this thread's early prefilter on ``stream`` (EarlyPrefilter): a
    consumer that waits on a later record of `done` waits on a later point of the same stream, so
    reuse never waits too little."""
    ev = getattr(_count_read, "pf_events", None)
    if ev is None:
        ev = _count_read.pf_events = {}
    e = ev.get(stream.cuda_stream)
    if e is None:
        e = ev[stream.cuda_stream] = (torch.cuda.Event(), torch.cuda.Event())
    return e


class EarlyPrefilter:
    """The literal prefilter launched before the line index is known on the host (it reads only
    the text): gram hits + the arena counters, handed to ``match_and_hits``."""

    def __init__(self, text, nbytes: int, tabs: dict, arena: "MatchArena", pf_grid: int, nlp=None,
                 stream: Optional["torch.cuda.Stream"] = None):
        L_est = int(nbytes * _LINES_PER_BYTE[0]) + 1
        self.cap = arena.caps(L_est)["gram"]
        self.gh = torch.empty(self.cap, dtype=torch.int64, device=text.device)
        self.cnt = torch.zeros(7, dtype=torch.int64, device=text.device)
        self.done = None
        st = _s(text)
        if stream is not None and nlp is None and text.is_cuda:
            # on its own stream: the rest of the line index (line starts / lengths, after the host's
            # line-count read) and the literal-free scans run beside it; match_and_hits waits for
            # `done` before the candidates' verification (config 2: the chains overlap)
            # (this thread's two events of this stream, reused)
            fork, done = _pf_events(stream)
            fork.record(torch.cuda.current_stream(text.device))
            stream.wait_event(fork)
            st = stream.cuda_stream
        N.prefilter_dev(text.data_ptr(), nbytes, tabs["pf"], 0, 0, self.gh.data_ptr(), self.cap, self.cnt.data_ptr(),
                        pf_grid, st, nlp)
        if st != _s(text):
            self.done = done
            self.done.record(stream)
            for t in (self.gh, self.cnt, text):     # (allocator bookkeeping: after the launch)
                t.record_stream(stream)


def match_and_hits(text, nbytes: int, line_start, line_len, tabs: dict, R: int, evt: tuple, arena: MatchArena,
                   ws: Optional[Workspace], pf_grid: int, scan_grid, timings=None, tick=None, side=None,
                   early: Optional[EarlyPrefilter] = None, defer: bool = False,
                   inject: Optional[torch.Tensor] = None, host_side=None):
    """GPU: every matcher appends to the arena, then the post-match hit pipeline reads the device
    counters itself -> (hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne) with ONE host read.

    ``defer``: no read -> (hits, hit_line, hit_off, ev_cnt, ev_end, hit capacity, device counters
    [gram, cand, ver, nh, ne], capacities incl. "ev"); the caller checks the counters against the
    capacities later (``MatchArena.overflow``) and re-runs with ``arena.learn``.

    ``side`` = (stream, fork event, join event): the self-verifying engines (literal-free DFA scan,
    single-DFA scan, MFMA NFA) run on that stream, concurrently with the literal prefilter chain
    (block index -> prefilter -> verify) on the current one; both join before the hit pipeline.
    A small request's kernels are latency-bound and leave most CUs idle, so the two chains
    overlap almost fully.

    ``inject``: device keys verified elsewhere (the host backtracker's side path,
    ``Engine.host_hits``), appended to the verified-hit buffer like a self-verifying engine's.

    ``host_side`` = (ops.side_path.HostSide, host bytes): the backtracker regexes fed by their
    relaxed automata export their device candidates to the host and get the verified keys back,
    all queued (side_path.hip); without it their device keys are only dropped (the host side path
    ran for them before, ``inject``)."""
    dev = text.device
    L = line_start.numel()
    st = _s(text)
    lbits, rbits = N.bits_for(max(L, 1)), N.bits_for(max(R, 1))
    scans = bool(tabs["scan_passes"]) or bool(tabs["scan_regs"].numel()) or \
        any(g.numel() for g in tabs["nfa_scan_lists"].values())
    ninj = 0 if inject is None else inject.numel()
    for attempt in range(8):         # each overflow learns the exact rates: one re-run is the rule
        cap = arena.caps(L)
        cap["ver"] += ninj
        early_done = None
        if early is not None:            # prefilter already queued (behind the line index)
            cap["gram"] = early.cap
            gh, cnt = early.gh, early.cnt
            early_done = early.done
        else:
            gh = torch.empty(cap["gram"], dtype=torch.int64, device=dev)
            # [gram hits, candidates, verified hits] then [unique hits, events] (post_hits counters),
            # then the events that fit their buffer (deferred steps: post_events' ne_fit) and the
            # DP step's overflow veto (k_dp_carry)
            cnt = torch.zeros(7, dtype=torch.int64, device=dev)
        cand = torch.empty(cap["cand"], dtype=torch.int64, device=dev)
        ver = torch.empty(cap["ver"], dtype=torch.int64, device=dev)
        c0 = cnt.data_ptr()
        sst = st
        if side is not None and scans and tick is None:
            side[1].record()
            side[0].wait_event(side[1])
            sst = side[0].cuda_stream
        blk = line_block_index(line_start, nbytes)
        # the long pole first: literal-free scans (own stream when `side`)
        for sp in tabs["scan_passes"]:
            N.scan_multi(text.data_ptr(), nbytes, line_start.data_ptr(), line_len.data_ptr(), L, sp, ver.data_ptr(),
                         cap["ver"], c0 + 16, scan_grid(sp), sst, True)
        if tabs["scan_regs"].numel():
            N.scan_dev(text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(), L, tabs["scan_regs"].data_ptr(),
                       tabs["scan_regs"].numel(), tabs["dfa"], ver.data_ptr(), cap["ver"], c0 + 16, sst)
        for ncls, glist in tabs["nfa_scan_lists"].items():
            if glist.numel():
                N.nfa(tabs["nfa_tables"].data_ptr(), glist.data_ptr(), glist.numel(), ncls, 0, L, text.data_ptr(),
                      line_start.data_ptr(), line_len.data_ptr(), 0, ver.data_ptr(), cap["ver"], c0 + 16, sst, True)
        if host_side is not None:          # region B: the scans' relaxation keys leave as the scans end
            host_side[0].begin(host_side[1])
            host_side[0].export_scan(ver, c0 + 16, cap["ver"], text, line_start, line_len, tabs["dfa"], sst)
        if sst != st:
            side[2].record(side[0])
        elif tick:
            tick("scan")
        if early is None:
            N.prefilter_dev(text.data_ptr(), nbytes, tabs["pf"], line_start.data_ptr(), L, gh.data_ptr(), cap["gram"],
                            c0, pf_grid, st)
        early = None                     # an overflow re-run launches everything itself
        if early_done is not None:       # the early prefilter ran on its own stream
            torch.cuda.current_stream(dev).wait_event(early_done)
        N.pf_verify_dev(gh.data_ptr(), cap["gram"], text.data_ptr(), nbytes, tabs["pf"], line_start.data_ptr(), L,
                        blk.data_ptr(), cand.data_ptr(), cap["cand"], c0 + 8, st, c0,
                        max(16, min(8192, nbytes >> 13)))
        if tick:
            tick("prefilter")
        if host_side is not None:          # region A: the prefilter candidates, right after the literal chain
            host_side[0].export_candidates(cand, c0 + 8, cap["cand"], text, line_start, line_len, tabs["dfa"], st)
        if sst != st:
            torch.cuda.current_stream(dev).wait_event(side[2])
        if host_side is not None:          # host backtracker answers for both regions -> append, all queued
            host_side[0].wait(ver, c0 + 16, cap["ver"], st)
        elif tabs.get("host_dev"):         # relaxation keys of regexes the host side path decided
            N.take_host(cand.data_ptr(), c0 + 8, cap["cand"], ver.data_ptr(), c0 + 16, cap["ver"], text.data_ptr(),
                        line_start.data_ptr(), line_len.data_ptr(), tabs["dfa"], None, st)
        if ninj:                           # (after the take: these keys are decided, never dropped)
            N.append_keys(ver.data_ptr(), cap["ver"], c0 + 16, inject.data_ptr(), ninj, st)
        n = cap["cand"] + cap["ver"]
        hits = torch.empty(n, dtype=torch.int64, device=dev)
        hit_line = torch.empty(n, dtype=torch.int32, device=dev)
        hit_off = torch.empty(R + 1, dtype=torch.int64, device=dev)
        ev_cnt = torch.empty(n, dtype=torch.int64, device=dev)
        ev_end = torch.empty(n, dtype=torch.int64, device=dev)

        def call(wp, wn):
            return N.post_hits(cand.data_ptr(), n, cap["cand"], lbits, rbits, R, text.data_ptr(),
                               line_start.data_ptr(), line_len.data_ptr(), tabs["dfa"], evt, hits.data_ptr(),
                               hit_line.data_ptr(), hit_off.data_ptr(), ev_cnt.data_ptr(), ev_end.data_ptr(),
                               c0 + 24, wp, wn, st, True, ver.data_ptr(), c0 + 8)

        _run_ws(call, ws)
        if defer:
            return hits, hit_line, hit_off, ev_cnt, ev_end, n, cnt, cap
        g, k, v, nh, ne = cnt[:5].tolist()             # the one host read
        arena.last = {"lines": L, "gram_hits": g, "prefilter_candidates": k, "scan_hits": v, "hits": nh, "events": ne}
        ok = g <= cap["gram"] and k <= cap["cand"] and v <= cap["ver"]
        arena.learn(L, {"gram": g, "cand": k, "ver": v}, overflow=not ok)
        if ok:
            return hits[:nh], hit_line, hit_off, ev_cnt, ev_end, nh, ne
        if host_side is not None:          # the worker answers every job before the re-run's export
            if host_side[0].settle() == 1:  # the GPU stopped waiting: the caller re-runs host-verified
                raise SidePathTimeout()
    raise RuntimeError(f"matching: buffers still overflowing after 8 attempts ({arena.last})")


class SidePathTimeout(RuntimeError):
    """The GPU's wait for the backtracker side path's host answer timed out (ops/side_path.py):
    the batch re-runs on the host-verified path (``Engine.prepare``)."""


def results_buffer(ne: int, nkeys: int, device) -> torch.Tensor:
    """One device buffer for everything a batch returns to the host (one D2H, no cat):
    [score f64 x ne | frequency counts i64 x max(nkeys, 1) | line i32 x ne | pattern i32 x ne |
    segment i32 x ne]."""
    return torch.empty(20 * ne + 8 * max(nkeys, 1), dtype=torch.uint8, device=device)


def results_views(buf: torch.Tensor, ne: int, nkeys: int):
    """(score, freq_counts, ev_line, ev_pat, ev_seg) views of ``results_buffer``."""
    k = max(nkeys, 1)
    a, b = 8 * ne, 8 * ne + 8 * k
    return (buf[:a].view(torch.float64), buf[a:b].view(torch.int64), buf[b:b + 4 * ne].view(torch.int32),
            buf[b + 4 * ne:b + 8 * ne].view(torch.int32), buf[b + 8 * ne:b + 12 * ne].view(torch.int32))


def post_events(hits, nh: int, ev_cnt, ev_end, ne: int, L: int, evt: tuple, text, line_start, line_len, dfa_tuple,
                nkeys: int, ws: Optional[Workspace], features: bool = True, ctx_ext: Tuple[int, int] = (1 << 30, 1 << 30),
                out: Optional[torch.Tensor] = None, dcounts: Optional[torch.Tensor] = None,
                ne_fit: Optional[torch.Tensor] = None):
    """Events in reference order + segment, frequency rank/key, per-key counts and context features
    (or, with ``features=False``, the int32 window coverage per line for another feature engine).
    ``ctx_ext`` = table extents of the 4 context DFAs (trans, acc entries) for LDS staging.
    ``out``: a ``results_buffer`` receiving line / pattern / segment / frequency counts.
    ``dcounts``: device [hits, events] counts (device only); nh / ne are then capacities and the
    outputs are left unset when the events exceed ne (the caller re-runs). ``ne_fit`` (int64[1],
    with ``dcounts``): receives the event count, or 0 when the events did not fit -- the count the
    batch's later kernels must read (score, summary), so they never touch unset event fields."""
    dev = text.device
    if out is not None:
        _, freq_counts, ev_line, ev_pat, ev_seg = results_views(out, ne, nkeys)
    else:
        ev_line = torch.empty(ne, dtype=torch.int32, device=dev)
        ev_pat = torch.empty(ne, dtype=torch.int32, device=dev)
        ev_seg = torch.empty(ne, dtype=torch.int32, device=dev)
        freq_counts = (torch.empty if nkeys else torch.zeros)(max(nkeys, 1), dtype=torch.int64, device=dev)
    ev_rank = torch.empty(ne, dtype=torch.int64, device=dev)
    ev_fkey = torch.empty(ne, dtype=torch.int64, device=dev)
    if out is not None and not nkeys:
        freq_counts.zero_()
    # k_feat_cov writes every line (0 outside windows); the host twin too
    feat = torch.empty(max(L, 1), dtype=torch.uint8, device=dev) if features and L else \
        torch.zeros(max(L, 1), dtype=torch.uint8, device=dev)
    cov = None if features else torch.zeros(max(L, 1), dtype=torch.int32, device=dev)
    lbits = N.bits_for(max(L, 1))

    def call(wp, wn):
        return N.post_events(hits.data_ptr() if nh else 0, nh, ev_cnt.data_ptr(), ev_end.data_ptr(), ne, L, lbits,
                             evt, text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(), dfa_tuple,
                             ev_line.data_ptr(), ev_pat.data_ptr(), ev_seg.data_ptr(), ev_rank.data_ptr(),
                             ev_fkey.data_ptr(), freq_counts.data_ptr(), feat.data_ptr() if features else 0,
                             _p(cov), ctx_ext[0], ctx_ext[1], wp, wn, _s(text), text.is_cuda, _p(dcounts),
                             _p(ne_fit))

    if text.is_cuda:
        _run_ws(call, ws)
    else:
        call(0, 0)
    return ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_counts, feat, cov


SUMMARY_MAX_K = 1024


def _check_k(k: int) -> None:
    """The summary kernel keeps at most SUMMARY_MAX_K rows: a larger top-k is a configuration
    error, not something to truncate silently (engine.topk is validated at config load)."""
    if int(k) > SUMMARY_MAX_K:
        raise ValueError(f"top-k {k} exceeds the summary kernel's maximum of {SUMMARY_MAX_K}")


def summarize(score: torch.Tensor, pat: torch.Tensor, line: torch.Tensor, k: int, sev_index: torch.Tensor,
              npat: int, nsev: int, line_add: Optional[torch.Tensor] = None, ws: Optional[Workspace] = None,
              pack_events: bool = False, hist_out: Optional[torch.Tensor] = None,
              rows_out: Optional[torch.Tensor] = None, dn: Optional[torch.Tensor] = None):
    """Top-k rows + histograms of scored events (csrc/kernels/summarize.hip).

    ``line`` is int32 (local, plus the device scalar ``line_add``) or int64 (global);
    ``sev_index[p]`` is pattern p's index into the library's distinct severity names. Returns
    (rows float64[k, 3] = (score, global line, pattern) ordered score desc, line asc, pattern asc,
    missing rows = (-inf, -1, -1); pat_hist int64[npat]; sev_hist int64[nsev]; packed) where
    ``packed`` (with ``pack_events``) is every event as uint8[20 n] = [global line int64 x n |
    score f64 x n | pattern int32 x n], written by the same kernel. No host sync. ``dn``: device
    event count (the arrays are capacities; ``packed`` then holds the events at stride *dn)."""
    dev = score.device
    _check_k(k)
    k = max(1, int(k))
    n = score.numel()
    rows = rows_out if rows_out is not None else torch.empty((k, 3), dtype=torch.float64, device=dev)
    if hist_out is not None:           # zeroed by the caller: [pattern hist | severity hist | ...]
        pat_hist, sev_hist = hist_out[:npat], hist_out[npat:npat + nsev]
    else:
        hist = torch.zeros(npat + nsev + 1, dtype=torch.int64, device=dev)
        pat_hist, sev_hist = hist[:npat], hist[npat:npat + nsev]
    packed = torch.empty(20 * n, dtype=torch.uint8, device=dev) if pack_events else None
    sev_of_pat = sev_index
    l32 = line.data_ptr() if line.dtype == torch.int32 else 0
    l64 = line.data_ptr() if line.dtype == torch.int64 else 0
    ins = (score.data_ptr() if n else 0, pat.data_ptr() if n else 0, l32 if n else 0, l64 if n else 0,
           _p(line_add), sev_of_pat.data_ptr(), 0, _p(packed) if n else 0, _p(dn))

    def call(wp, wn):
        return N.summarize(ins, n, k, nsev, rows.data_ptr(), pat_hist.data_ptr(), sev_hist.data_ptr(), wp, wn, _s(score),
                           score.is_cuda)

    if score.is_cuda:
        _run_ws(call, ws if ws is not None else Workspace(dev))
    else:
        call(0, 0)
    return rows, pat_hist[:npat], sev_hist[:nsev], packed


def dp_payload_width(nk: int, ns: int) -> int:
    """Columns of the C1+C3+C4 all-gather payload: owned lines, nk counts, ns chain slots, overflow."""
    return 1 + nk + ns + 1


def dp_pack(own_lines: int, freq_counts: torch.Tensor, nk: int, chain: torch.Tensor,
            out: Optional[torch.Tensor] = None, overflow: Optional[tuple] = None) -> torch.Tensor:
    """C1+C3+C4 all-gather payload [owned lines | nk frequency counts | chain table | overflow flag]
    (int64); ``out``: where to write it (this rank's row of an in-place all-gather buffer);
    ``overflow`` = (device counters [5], host capacities [4]) of a deferred-count step: the flag is
    set when a counter exceeded its buffer (every rank then vetoes the step's record and re-runs)."""
    ns = chain.numel()
    pack = out if out is not None else torch.empty(dp_payload_width(nk, ns), dtype=torch.int64, device=chain.device)
    fc = freq_counts if freq_counts.dtype == torch.int64 else freq_counts.to(torch.int64)
    cnt, caps = (overflow[0].data_ptr(), [int(c) for c in overflow[1]]) if overflow is not None else (0, [])
    N.dp_pack(int(own_lines), fc.data_ptr(), nk, chain.data_ptr(), ns, pack.data_ptr(), _s(chain), chain.is_cuda,
              cnt, caps)
    return pack


def dp_carry(g: torch.Tensor, rank: int, nk: int, ns: int, halo_left: int, tot: Optional[torch.Tensor],
             slot_e0: torch.Tensor, slot_k: torch.Tensor, red_tail: Optional[torch.Tensor] = None,
             veto_out: Optional[torch.Tensor] = None, zero: Optional[torch.Tensor] = None,
             stream: Optional[tuple] = None):
    """From the gathered payloads: (own_start[1], g0[1], n[1], carry[nk], seq_carry uint8[ns],
    veto[1]); ``red_tail`` (optional) receives this rank's frequency counts; veto = any rank's
    overflow flag (written into ``veto_out`` when given); ``zero`` (int64, optional) is zeroed by
    the same kernel. ``stream`` = (seq_base uint8[ns], line_base, n_fixed, seq_next uint8[ns]): one
    step of a stream of steps (the earlier steps' sequence state and line count, an open N, and the
    sequence state after this step written into seq_next)."""
    dev = g.device
    sc = torch.empty(5, dtype=torch.int64, device=dev)          # own_start, g0, n, veto (+ pad)
    carry = torch.empty(max(nk, 1), dtype=torch.int64, device=dev)
    if nk == 0:
        carry.zero_()
    seq = torch.empty(max(ns, 1), dtype=torch.uint8, device=dev)
    g = g.contiguous()
    p = sc.data_ptr()
    veto = veto_out if veto_out is not None else sc[3:4]
    args = (g.data_ptr(), g.shape[0], rank, nk, ns, int(halo_left), _p(tot) if nk else 0, slot_e0.data_ptr(),
            slot_k.data_ptr(), p, p + 8, p + 16, carry.data_ptr(), seq.data_ptr(), _p(red_tail), veto.data_ptr(),
            _p(zero), 0 if zero is None else zero.numel())
    if stream is not None:
        sb, lb, nf, sn = stream
        args = args + (_p(sb), int(lb), int(nf), _p(sn))
    N.dp_carry(args, _s(g), g.is_cuda)
    return sc[0:1], sc[1:2], sc[2:3], carry, seq, veto


def topk_rows(rows: torch.Tensor, k: int, ws: Optional[Workspace] = None) -> torch.Tensor:
    """Merge (score, line, pattern) rows (e.g. every rank's top-k) into the k best, same order."""
    dev = rows.device
    _check_k(k)
    k = max(1, int(k))
    rows = rows.contiguous()
    out = torch.empty((k, 3), dtype=torch.float64, device=dev)
    ins = (0, 0, 0, 0, 0, 0, rows.data_ptr())

    def call(wp, wn):
        return N.summarize(ins, rows.shape[0], k, 0, out.data_ptr(), 0, 0, wp, wn, _s(rows), rows.is_cuda)

    if rows.is_cuda:
        _run_ws(call, ws if ws is not None else Workspace(dev))
    else:
        call(0, 0)
    return out


def rescore(gl: torch.Tensor, fac: torch.Tensor, n_lines: int, sp_tuple) -> torch.Tensor:
    """Final streaming scores: the score kernel's kept factors with the chronological factor of the
    true global line count (left-to-right product, ScoringService.java:102-109)."""
    n = gl.numel()
    out = torch.empty(n, dtype=torch.float64, device=gl.device)
    if n:
        N.rescore(gl.data_ptr(), fac.contiguous().data_ptr(), n, int(n_lines), sp_tuple, out.data_ptr(), _s(gl),
                  gl.is_cuda)
    return out


def score_fused(ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_carry, st_tuple, sp_tuple, with_factors=False,
                out: Optional[torch.Tensor] = None, dn: Optional[torch.Tensor] = None):
    """k_score with the frequency count fused in: freq = carry[fkey] + rank (-1 without a key).
    ``out``: float64[n] destination (e.g. the score view of a ``results_buffer``); ``dn``: device
    event count (the arrays are then capacities; device only)."""
    n = ev_line.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=ev_line.device)
    fac = torch.empty((n, 7), dtype=torch.float64, device=ev_line.device) if with_factors else None
    if n == 0:
        return out, fac
    args = (ev_line.data_ptr(), ev_pat.data_ptr(), ev_seg.data_ptr(), ev_rank.data_ptr(), ev_fkey.data_ptr(),
            freq_carry.data_ptr(), n, st_tuple, sp_tuple, out.data_ptr(), _p(fac))
    if ev_line.is_cuda:
        N.score_dev(*args, _s(ev_line), _p(dn))
    else:
        N.score_host(*args)
    return out, fac
