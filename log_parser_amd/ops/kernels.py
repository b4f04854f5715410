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


def newline_positions(text: torch.Tensor, nbytes: int, flag_cr: bool = False) -> torch.Tensor:
    """Positions of every '\\n' in text[0:nbytes] (int64, ascending). ``flag_cr`` (device only):
    bit 62 marks a '\\n' preceded by '\\r' -- the input format of ``lines_dev``."""
    if text.is_cuda:
        nb = N.nl_tiles(nbytes)
        if nb == 0:
            return torch.empty(0, dtype=torch.int64, device=text.device)
        cnt = torch.empty(nb, dtype=torch.int32, device=text.device)
        N.nl_count_dev(text.data_ptr(), nbytes, cnt.data_ptr(), _s(text))
        off = torch.cumsum(cnt, 0, dtype=torch.int64)
        total = int(off[-1].item())
        off = off - cnt.to(torch.int64)
        pos = torch.empty(total, dtype=torch.int64, device=text.device)
        N.nl_write_dev(text.data_ptr(), nbytes, off.data_ptr(), pos.data_ptr(), int(flag_cr), _s(text))
        return pos
    c = N.nl_positions_host(text.data_ptr(), nbytes, 0)
    pos = torch.empty(c, dtype=torch.int64)
    N.nl_positions_host(text.data_ptr(), nbytes, pos.data_ptr())
    return pos


def split_lines(text: torch.Tensor, nbytes: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Java ``logs.split("\\\\r?\\\\n")`` line index (AnalysisService.java:53).

    Returns (line_start int64[L], line_len int32[L]); trailing empty lines removed; input
    without any newline is one line (possibly empty).
    """
    dev = text.device
    nl = newline_positions(text, nbytes, flag_cr=text.is_cuda)
    if nl.numel() == 0:
        return (torch.zeros(1, dtype=torch.int64, device=dev),
                torch.full((1,), nbytes, dtype=torch.int32, device=dev))
    if text.is_cuda:                       # k_lines (CR flags from k_nl_write) + k_last_nonempty
        n = nl.numel()
        starts = torch.empty(n + 1, dtype=torch.int64, device=dev)
        lens = torch.empty(n + 1, dtype=torch.int32, device=dev)
        last = torch.zeros(1, dtype=torch.int64, device=dev)
        N.lines_dev(nl.data_ptr(), n, text.data_ptr(), nbytes, starts.data_ptr(), lens.data_ptr(), last.data_ptr(),
                    _s(text))
        L = int(last.item())
        return starts[:L], lens[:L]
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
    nl = newline_positions(text, nbytes)
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


LINE_BLK_SHIFT = 12


def line_block_index(line_start: torch.Tensor, nbytes: int) -> torch.Tensor:
    """blk[b] = line containing byte b << 12 (int32), for O(log lines-per-4KiB) line lookups."""
    nblk = (max(nbytes, 1) >> LINE_BLK_SHIFT) + 2
    pos = torch.arange(nblk, dtype=torch.int64, device=line_start.device) << LINE_BLK_SHIFT
    idx = torch.searchsorted(line_start, pos, right=True) - 1
    return idx.clamp(min=0).to(torch.int32)


def prefilter(text, nbytes, pf_tuple, line_start, cap: int, grid: int = 2048) -> torch.Tensor:
    """Literal prefilter -> (regex << 32 | line) candidates.

    GPU: k_prefilter streams the text and stages bloom gram hits (position, gram length);
    k_pf_verify then checks whole literals, one lane per hit (keeps the streaming kernel tight).
    """
    nlines = line_start.numel()
    if text.is_cuda:
        gcap = cap
        while True:
            gh = torch.empty(max(gcap, 1), dtype=torch.int64, device=text.device)
            cnt = torch.zeros(1, dtype=torch.int64, device=text.device)
            N.prefilter_dev(text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(), nlines, gh.data_ptr(), gcap,
                            cnt.data_ptr(), grid, _s(text))
            c = int(cnt.item())
            if c <= gcap:
                gh = gh[:c]
                break
            gcap = c
        if gh.numel() == 0:
            return torch.empty(0, dtype=torch.int64, device=text.device)
        blk = line_block_index(line_start, nbytes)
        while True:
            cand = torch.empty(max(cap, 1), dtype=torch.int64, device=text.device)
            cnt = torch.zeros(1, dtype=torch.int64, device=text.device)
            N.pf_verify_dev(gh.data_ptr(), gh.numel(), text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(),
                            nlines, blk.data_ptr(), cand.data_ptr(), cap, cnt.data_ptr(), _s(text))
            c = int(cnt.item())
            if c <= cap:
                return cand[:c]
            cap = c
    while True:
        cand = torch.empty(max(cap, 1), dtype=torch.int64)
        c = N.prefilter_host(text.data_ptr(), nbytes, pf_tuple, line_start.data_ptr(), nlines, cand.data_ptr(), cap)
        if c <= cap:
            return cand[:c]
        cap = c


def verify(cand, text, line_start, line_len, dfa_tuple) -> torch.Tensor:
    out = torch.empty(cand.numel(), dtype=torch.uint8, device=cand.device)
    if cand.numel() == 0:
        return out
    if cand.is_cuda:
        N.verify_dev(cand.data_ptr(), cand.numel(), text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(),
                     dfa_tuple, out.data_ptr(), _s(cand))
    else:
        N.verify_host(cand.data_ptr(), cand.numel(), text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(),
                      dfa_tuple, out.data_ptr())
    return out


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


def context_features(lines: torch.Tensor, L: int, text, line_start, line_len, dfa_tuple) -> torch.Tensor:
    """uint8 feature bits per line (ERR 1, WARN 2, STACK 4, EXC 8) for the given line ids; 0 elsewhere."""
    feat = torch.zeros(max(L, 1), dtype=torch.uint8, device=text.device)
    if lines.numel():
        N.feat(lines.data_ptr(), lines.numel(), text.data_ptr(), line_start.data_ptr(), line_len.data_ptr(),
               dfa_tuple, feat.data_ptr(), _s(text), text.is_cuda)
    return feat


def score(ev_line, ev_pat, ev_seg, ev_freq, st_tuple, sp_tuple, with_factors: bool = False):
    n = ev_line.numel()
    out = torch.empty(n, dtype=torch.float64, device=ev_line.device)
    fac = torch.empty((n, 7), dtype=torch.float64, device=ev_line.device) if with_factors else None
    if n == 0:
        return out, fac
    if ev_line.is_cuda:
        N.score_dev(ev_line.data_ptr(), ev_pat.data_ptr(), ev_seg.data_ptr(), ev_freq.data_ptr(), n, st_tuple,
                    sp_tuple, out.data_ptr(), _p(fac), _s(ev_line))
    else:
        N.score_host(ev_line.data_ptr(), ev_pat.data_ptr(), ev_seg.data_ptr(), ev_freq.data_ptr(), n, st_tuple,
                     sp_tuple, out.data_ptr(), _p(fac))
    return out, fac


def nfa_features(groups: torch.Tensor, lines: torch.Tensor, L: int, text, line_start, line_len,
                 group_list: torch.Tensor, ncls: int) -> torch.Tensor:
    """Context features via the MFMA NFA kernel (group 0 = the 4 context regexes): uint8 bits per line."""
    feat = torch.zeros(max(L, 1), dtype=torch.uint8, device=text.device)
    if lines.numel():
        N.nfa(groups.data_ptr(), group_list.data_ptr(), 1, ncls, lines.data_ptr(), lines.numel(), text.data_ptr(),
              line_start.data_ptr(), line_len.data_ptr(), feat.data_ptr(), 0, 0, 0, _s(text), text.is_cuda)
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
