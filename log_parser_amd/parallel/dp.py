"""Line-sharded data parallelism over the GPUs of one node (RCCL over xGMI).

The reference is single-threaded per request; this module is new. One logical log
is split into contiguous line ranges, one per rank (one process per GPU), each with ``H`` halo
lines on both sides (``H = CompiledLibrary.halo`` = max of proximity window, context lines and
the ±5 sequence window). Every cross-shard dependency of the reference's sequential semantics is
resolved with collectives:

  C1  global N / line offsets  (ScoringService.java:125)      \\
  C3  frequency ordering       (ScoringService.java:84-88)     } in-place all_gather #1, int64
  C4  backward sequence chain  (ScoringService.java:296-305)  /   [own_lines | freq counts | chain]
  C5/C6 severity histogram + frequency histogram  \  in-place all_gather #2 of
  C7  top-k events                                /   [pattern hist | severity hist | freq counts | k rows],
                                                     then a local sum over ranks + top-k merge
  (the local halves of C5-C7 are one hand-written kernel chain, csrc/kernels/summarize.hip)

Two collectives per step, both in place (this rank's payload is written straight into its row of
the gather buffer): at world size 1 RCCL moves no bytes at all -- a world-1 copy was the
self-copy that queued behind the PCIe ingest in round 2 -- and at world size N each step moves
N x ~20 KB, latency-bound either way (an all-reduce would be the same number of latency hops and
the top-k rows have to be gathered anyway).
  C2  halos: by default every rank stages its halo lines from the shared host source together
      with its own lines (no extra collective); ``exchange_halos`` is the point-to-point variant
      (batch_isend_irecv with both neighbours) for ranks that only hold their own lines

xGMI bandwidth is irrelevant here; PCIe ingest and HBM are what scale. The backend is whatever
``torch.distributed`` was initialised with: ``nccl`` (= RCCL on ROCm) on GPUs, ``gloo`` for the
CPU tests (and to rehearse several ranks on one GPU, host-staged).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine import Engine, RunResult, Segments, summary_from_severity
from ..ops import kernels as K


def world() -> tuple:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def host_staged(group=None) -> bool:
    """True when the process group cannot move device tensors (gloo): collectives then stage
    through host memory. Production GPU runs use nccl (= RCCL) and never take this path; it lets
    the multi-rank GPU pipeline be exercised with several ranks on ONE GPU (tests/test_dp.py)."""
    return dist.get_backend(group) == "gloo"


def distributed() -> bool:
    """A process group exists. Collectives then always run -- also at world size 1 (the bench's
    default on a GPU is a world-1 RCCL group, so the 1-GPU number drives the same calls the
    8-GPU run makes; in place, they move no bytes there)."""
    return dist.is_available() and dist.is_initialized()


def all_gather_inplace(buf: torch.Tensor, group=None) -> torch.Tensor:
    """In-place all_gather of ``buf`` [world, n]: this rank's row is already filled; on return
    every row is (RCCL all_gather_into_tensor with the input aliasing its output row)."""
    r, w = world()
    if not distributed():
        return buf
    if buf.is_cuda and not host_staged(group):
        dist.all_gather_into_tensor(buf, buf[r], group=group)
        return buf
    h = buf.cpu()
    rows = list(h.unbind(0))
    dist.all_gather(rows, h[r].clone(), group=group)
    buf.copy_(h)
    return buf


def all_gather_rows(t: torch.Tensor, group=None) -> torch.Tensor:
    """all_gather of a 1-D tensor -> [world, n] (RCCL all_gather_into_tensor on GPU)."""
    r, w = world()
    if not distributed():
        return t.unsqueeze(0)
    if t.is_cuda and not host_staged(group):
        out = torch.empty((w,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        return out
    src = t.detach().cpu().contiguous()
    out = torch.empty((w,) + tuple(t.shape), dtype=t.dtype)
    dist.all_gather(list(out.unbind(0)), src, group=group)
    return out.to(t.device)


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if distributed():
        if t.is_cuda and host_staged(group):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


@dataclass
class StreamCarry:
    """The carries of earlier steps when a long log is streamed as a sequence of DP steps
    (parallel/stream.py ShardedStreamAnalyzer) -- the same protocol as a chunk of one stream:
    the frequency carry (window totals at the stream's start + every earlier step's counts), the
    sequence-chain state before the step, and the global index of the step's first line. The
    chronological factor's N is open (the step keeps every event's factors; rescored at the end)."""
    freq: torch.Tensor             # int64 [max(nk, 1)]
    seq: torch.Tensor              # uint8 [max(ns, 1)]
    line_base: int = 0


@dataclass
class StepOutput:
    result: RunResult
    own_counts: torch.Tensor       # owned lines per rank (C1 all-gather), stays on the device
    rank: int
    pattern_counts: torch.Tensor   # global (all-reduced) events per pattern
    severity_counts: Optional[torch.Tensor] = None  # global events per library severity name
    # rank 0: merged global top-k rows (score, 0-based global line, pattern), score desc / line asc
    # / pattern asc, padded with (-inf, -1, -1) when fewer events exist; stays on the device
    topk_rows: Optional[torch.Tensor] = None
    own_lo: int = 0                                 # first owned local line (= left halo lines)
    own_start_dev: Optional[torch.Tensor] = None    # [1] global index of the first owned line
    # pack_events: every owned event as uint8[20 n] = [global line i64 | score f64 | pattern i32]
    events_packed: Optional[torch.Tensor] = None
    # GPU: recorded on the compute stream after the step's last kernel (before its count read)
    end_event: Optional[object] = None
    # stream steps: the sequence-chain state after the step and the step's summed frequency counts
    seq_next: Optional[torch.Tensor] = None
    freq_counts: Optional[torch.Tensor] = None

    # host integers on demand (a host read here would stall the step's launch queue)
    @property
    def total_lines(self) -> int:
        return int(self.own_counts.sum().item())

    @property
    def own_start(self) -> int:
        return int(self.own_counts[:self.rank].sum().item())

    def _top(self, col: int) -> Optional[torch.Tensor]:
        if self.topk_rows is None:
            return None
        r = self.topk_rows
        k = int(torch.isfinite(r[:, 0]).sum().item())
        return r[:k, col] if col == 0 else r[:k, col].to(torch.int64)

    @property
    def topk_score(self) -> Optional[torch.Tensor]:
        return self._top(0)

    @property
    def topk_line(self) -> Optional[torch.Tensor]:
        return self._top(1)

    @property
    def topk_pat(self) -> Optional[torch.Tensor]:
        return self._top(2)


class ShardedAnalyzer:
    def __init__(self, engine: Engine, group=None):
        self.engine = engine
        self.group = group
        self.time_reduce = False          # events around collective 2's local sum / top-k merge
        self._reduce_ev: list = []
        lib = engine.lib
        # per sequence-event slot: first slot of its sequence and its event index
        off = lib.seq_ev_off
        e0 = np.zeros(max(lib.n_seq_events, 1), np.int64)
        kk = np.zeros(max(lib.n_seq_events, 1), np.int64)
        for q in range(off.size - 1):
            e0[off[q]:off[q + 1]] = off[q]
            kk[off[q]:off[q + 1]] = np.arange(off[q + 1] - off[q])
        dev = engine.device
        self.slot_e0 = torch.from_numpy(e0).to(dev)
        self.slot_k = torch.from_numpy(kk).to(dev)

    def step(self, text: torch.Tensor, nbytes: int, ls: Optional[torch.Tensor], ll: Optional[torch.Tensor],
             halo_left: int, halo_right: int, topk: int = 100, with_factors: bool = False,
             pack_events: bool = False, stream_carry: Optional[StreamCarry] = None,
             split_trim: bool = True, host_text=None) -> StepOutput:
        """One shard step. ``ls`` / ``ll`` = None: the line index is built here, with the literal
        prefilter queued behind it before its host read (the GPU filters while the host waits).

        On a GPU the step reads NO counts between its matchers and its end: hits and events run in
        device-count mode on capacity-sized buffers (``Engine.prepare(defer=True)``), so the host
        queues the whole step -- event stage, both collectives, carry, score, summary, record --
        while the GPU is still matching. Each rank's overflow flag rides in collective 1; any
        overflow vetoes the frequency record on every rank, and after the one end-of-step read all
        ranks re-run the step with the capacities they learned.

        ``stream_carry``: the step is one of a stream of steps -- its carries come from the earlier
        steps, N stays open (factors kept, ``with_factors`` implied), the frequency window is not
        recorded (the stream records once, at its end) and the output carries the sequence state
        after the step and the step's summed frequency counts.

        ``host_text``: the shard's bytes in host memory (numpy view), read by the backtracker side
        path of a library with non-regular regexes instead of a device-to-host copy of the text."""
        eng = self.engine
        rank, wsize = world()
        early = None
        if ls is None:
            box = []
            if eng.fuses_line_index(text):      # the prefilter's read of the text also counts the lines
                ls, ll = K.split_lines(text, nbytes, fused=lambda nlp: box.append(eng.prefilter_early(text, nbytes, nlp)))
                early = box[0] if box else None
            else:
                ls, ll, early = eng.split_with_prefilter(text, nbytes)
        defer = eng.can_defer(text)
        for attempt in range(4):
            out, prep, veto = self._step(text, nbytes, ls, ll, halo_left, halo_right, topk,
                                         with_factors or stream_carry is not None, pack_events,
                                         early if attempt == 0 else None, defer, stream_carry, split_trim,
                                         host_text)
            if not defer:
                return out
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            h = prep.cnt.cpu().tolist()          # the step's one count read, at its end (veto = cnt[6])
            counts, L = h[:5], ls.numel()
            if not h[6]:
                eng.arena.learn_deferred(L, counts)
                out.end_event = end
                return self._trim(out, prep, counts[4])
            # some rank overflowed a buffer: every rank learns its exact rates and re-runs
            eng.arena.learn(L, {"gram": counts[0], "cand": counts[1], "ver": counts[2], "ev": counts[4]}, overflow=True)
            if eng._host_side is not None:      # the side path's worker answers before the re-run's export
                eng._host_side.settle()
        raise RuntimeError("DP step: buffers still overflowing after re-runs")

    @staticmethod
    def _trim(out: StepOutput, prep, ne: int) -> StepOutput:
        """A deferred step's capacity-sized event arrays cut to the step's ``ne`` events."""
        r = out.result
        r.ev_line, r.ev_pat, r.ev_seg, r.score = r.ev_line[:ne], r.ev_pat[:ne], r.ev_seg[:ne], r.score[:ne]
        if r.factors is not None:
            r.factors = r.factors[:ne]
        if out.events_packed is not None:
            out.events_packed = out.events_packed[:20 * ne]
        return out

    def _step(self, text, nbytes, ls, ll, halo_left, halo_right, topk, with_factors, pack_events, early, defer,
              sc: Optional[StreamCarry] = None, split_trim: bool = True, host_text=None):
        eng = self.engine
        lib = eng.lib
        rank, wsize = world()
        dev = text.device
        L = ls.numel()
        own_lo, own_hi = halo_left, L - halo_right
        segs = Segments.scalar(0, L, own_lo, own_hi, 0, 1, dev, upload=eng.upload)
        prep = eng.prepare(text, nbytes, ls, ll, segs, early=early, defer=defer, split_trim=split_trim,
                           host_text=host_text)
        chain = eng.seq_chain_table(prep, own_lo, own_hi)
        nk = len(lib.freq_ids)
        ns = chain.numel()
        g = torch.empty((wsize, K.dp_payload_width(nk, ns)), dtype=torch.int64, device=dev)
        ovf = None
        if defer:
            c = prep.caps
            ovf = (prep.cnt, (c["gram"], c["cand"], c["ver"], c["ev"]))
        K.dp_pack(own_hi - own_lo, prep.freq_counts, nk, chain, out=g[rank], overflow=ovf)   # k_dp_pack -> own row
        all_gather_inplace(g, self.group)                          # collective 1: C1 + C3 + C4 + overflow
        own_counts = g[:, 0]
        # collective 2 buffer, one row per rank: [pattern hist | severity hist | frequency counts |
        # top-k rows (k x 3 f64)]; k_dp_carry seeds the counts, the summary kernel the histograms + rows
        P, S = len(lib.patterns), len(lib.sev_names)
        K._check_k(topk)
        k = max(1, topk)
        H = P + S + nk
        red2 = torch.empty((wsize, H + 3 * k), dtype=torch.int64, device=dev)   # other rows: the all-gather
        mine = red2[rank]
        seq_next = None
        stream = None
        if sc is not None:
            seq_next = torch.empty(max(ns, 1), dtype=torch.uint8, device=dev)
            stream = (sc.seq, sc.line_base, 1 << 62, seq_next)
        own_start, segs.g0, segs.n, carry, seq_carry, veto = K.dp_carry(     # k_dp_carry: device scalars, no sync
            g, rank, nk, ns, halo_left, (sc.freq if sc is not None else eng.freq_carry()) if nk else None,
            self.slot_e0, self.slot_k, red_tail=mine[P + S:H] if nk else None,
            veto_out=prep.cnt[6:7] if defer else None, zero=mine[:P + S],   # histogram slots (summary kernel adds)
            stream=stream)
        res = eng.finish(prep, segs, carry, seq_carry, with_factors)
        # C5/C6 + C7 local half: one summarize kernel chain (pattern + severity histograms and this
        # rank's top-k rows with global line numbers, no host sync) into this rank's row
        rows_out = mine[H:].view(torch.float64).view(k, 3)
        _, _, _, packed = K.summarize(res.score, res.ev_pat, res.ev_line, k, eng.tabs["sev_index"], P, S,
                                      line_add=segs.g0, ws=eng.ws, pack_events=pack_events, hist_out=mine[:H],
                                      rows_out=rows_out, dn=prep.ne_dev)
        all_gather_inplace(red2, self.group)                       # collective 2: C5 + C6 + C7
        tev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if self.time_reduce and dev.type == "cuda" else None
        if tev:
            tev[0].record()
        red = red2[:, :H].sum(0) if wsize > 1 else red2[0, :H]
        if tev:
            tev[1].record()
        if sc is None:
            eng.commit_frequency(red[P + S:], veto=veto if defer else None)
        out = StepOutput(res, own_counts, rank, red[:P], severity_counts=red[P:P + S], own_lo=own_lo,
                         own_start_dev=own_start, events_packed=packed, seq_next=seq_next,
                         freq_counts=red[P + S:H] if nk else None)
        if topk > 0 and rank == 0:
            allrows = red2[:, H:].contiguous().view(torch.float64).view(-1, 3)
            out.topk_rows = K.topk_rows(allrows, k, ws=eng.ws) if allrows.shape[0] > k else allrows
        if tev:
            tev[2].record()
            self._reduce_ev.append(tev)
        return out, prep, veto

    @property
    def reduce_us(self) -> list:
        """Per step with ``time_reduce``: (local sum over the [world, H] histogram rows, rank-0 top-k
        merge of world x k rows) in us, from events (read after the steps, no sync inside them)."""
        out = []
        for a, b, c in self._reduce_ev:
            c.synchronize()
            out.append((a.elapsed_time(b) * 1e3, b.elapsed_time(c) * 1e3))
        return out

    def summary(self, pattern_counts: torch.Tensor, first_pat: Optional[int] = None,
                severity_counts: Optional[torch.Tensor] = None) -> dict:
        """AnalysisSummary of a step (AnalysisService.java:188-215); from the severity histogram
        when given (S entries instead of P)."""
        lib = self.engine.lib
        if severity_counts is not None:
            sc = severity_counts.cpu().numpy()
        else:
            pc = pattern_counts.cpu().numpy()
            sc = np.bincount(lib.sev_index, weights=pc, minlength=len(lib.sev_names)).astype(np.int64)
        return summary_from_severity(lib, sc, first_pat)


def halo_bytes(data, n_lines: int) -> tuple:
    """(head, tail): byte length of the first / last ``n_lines`` lines of ``data`` (a shard made of
    complete '\\n'-terminated lines, the last rank's final line may be unterminated)."""
    n = len(data)
    head, pos = 0, 0
    for _ in range(n_lines):
        j = data.find(b"\n", pos)
        if j < 0:
            head = n
            break
        head = pos = j + 1
    end = n
    start = n
    for _ in range(n_lines):
        j = data.rfind(b"\n", 0, start - 1) if start > 0 else -1
        start = j + 1
        if start == 0:
            break
    return head, end - start


def exchange_halos(own: torch.Tensor, own_nbytes: int, head: int, tail: int, group=None):
    """C2: point-to-point halo exchange with the neighbour ranks (RCCL send/recv over
    one xGMI hop; gloo on CPU). Sends ``own[:head]`` (first H lines) to rank-1 and
    ``own[own_nbytes-tail:own_nbytes]`` (last H lines) to rank+1; returns (left, right) halos.
    Sizes travel first in one tiny all_gather so every receive is posted with its exact length."""
    r, w = world()
    dev = own.device
    if w == 1:
        z = torch.empty(0, dtype=torch.uint8, device=dev)
        return z, z
    sizes = all_gather_rows(torch.tensor([head, tail], dtype=torch.int64, device=dev), group).cpu()
    lsize = int(sizes[r - 1, 1]) if r > 0 else 0
    rsize = int(sizes[r + 1, 0]) if r < w - 1 else 0
    left = torch.empty(lsize, dtype=torch.uint8, device=dev)
    right = torch.empty(rsize, dtype=torch.uint8, device=dev)
    peer = (lambda x: dist.get_global_rank(group, x)) if group is not None else (lambda x: x)
    plan = []                                           # (isend | irecv, device tensor, peer)
    if r > 0 and head:
        plan.append((dist.isend, own[:head].contiguous(), peer(r - 1)))
    if r > 0 and lsize:
        plan.append((dist.irecv, left, peer(r - 1)))
    if r < w - 1 and tail:
        plan.append((dist.isend, own[own_nbytes - tail:own_nbytes].contiguous(), peer(r + 1)))
    if r < w - 1 and rsize:
        plan.append((dist.irecv, right, peer(r + 1)))
    if plan:
        staged = dev.type == "cuda" and host_staged(group)   # gloo p2p moves host tensors only
        bufs = [t.cpu() if staged else t for _, t, _ in plan]
        ops = [dist.P2POp(fn, b_, pr, group) for (fn, _, pr), b_ in zip(plan, bufs)]
        for q in dist.batch_isend_irecv(ops):
            q.wait()
        if staged:
            for (fn, t, _), b_ in zip(plan, bufs):
                if fn is dist.irecv:
                    t.copy_(b_)
    return left, right


def assemble_shard(own: torch.Tensor, own_nbytes: int, left: torch.Tensor, right: torch.Tensor):
    """[left halo | own | right halo | zero pad] as one padded device text + its line index and
    halo line counts (halo lines are complete, so they are counted by their '\\n's)."""
    from ..ops import kernels as K
    n = left.numel() + own_nbytes + right.numel()
    text = torch.zeros(K.padded_len(n), dtype=torch.uint8, device=own.device)
    a = left.numel()
    text[:a] = left
    text[a:a + own_nbytes] = own[:own_nbytes]
    text[a + own_nbytes:n] = right
    ls, ll = K.split_lines(text, n)
    hl = int((left == 10).sum().item()) if a else 0
    hr = 0
    if right.numel():
        hr = int((right == 10).sum().item()) + (0 if int(right[-1].item()) == 10 else 1)
    return text, n, ls, ll, hl, hr


def shard_bounds(n_lines: int, world_size: int, rank: int, halo: int):
    """Contiguous balanced line ranges; returns (lo, hi, halo_left, halo_right) in global lines."""
    base, rem = divmod(n_lines, world_size)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    hl = min(halo, lo)
    hr = min(halo, n_lines - hi)
    return lo, hi, hl, hr
