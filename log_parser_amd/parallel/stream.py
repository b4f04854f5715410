"""Long-log streaming ("sequence parallel" for logs; BASELINE config #4).

A log far larger than one request (100 GB, 1B lines) is processed in line-aligned chunks of
``engine.chunk-bytes``. A chunk is handled exactly like a data-parallel shard that runs after
all previous ones (parallel/dp.py), so the result equals the single-pass reference semantics:

* halos: ``CompiledLibrary.halo`` lines of the previous / next chunk are staged with each chunk
  (proximity ≤ max-window, context lines, ±5 sequence window);
* frequency: the running per-id match count of earlier chunks is the scan carry;
* backward sequence search: a running per-slot state composed with each chunk's chain table
  (``state'[j] = 1 if f[j] < 0 else state[slot(q, f[j])]``) replaces the unbounded scan;
* chronological factor: needs the total line count N, unknown until the end, so the chunk pass
  keeps every event's factors (k_score with factors) and the final pass recomputes
  ``conf*sev*chrono*prox*temp*ctx*(1-pen)`` in the reference's left-to-right order — one pass
  over the bytes, no re-read.

Ingest is pipelined: a host thread stages chunk k+1 into pinned memory while the GPU analyses
chunk k; the H2D copy runs on its own HIP stream.
"""
from __future__ import annotations

import queue
from collections import deque
import threading
import time
import warnings
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch

from ..engine import Engine, Segments
from ..ops import kernels as K
from ..utils.hostmem import registered_empty


CHUNK_MIN, CHUNK_MAX = 256 << 20, 8 << 30


def auto_chunk_bytes(device: torch.device, total: Optional[int] = None) -> int:
    """``engine.chunk-bytes = 0``: chunks sized from the GPU's free HBM -- 1/16 of it, within
    [256 MiB, 8 GiB] (a chunk's device footprint is ~3x its bytes: text, line index, matcher
    arenas, CSR, with the next chunk's copy in flight). On a 288 GB MI355X that is 8 GiB chunks:
    fewer halos, launches and host hand-offs than the 256 MiB of round 2 -- what a resident log
    (analysed from HBM, no copy to hide) wants. A host stream (``total`` = its length) also caps
    the chunk at 1/8 of the stream, so it still has a steady state between the ramps
    (``StreamAnalyzer._plan``: the ramps overlap the first copy and the last analysis; 1B lines
    with 8 GiB chunks ran at 526M lines/s, 256 MiB chunks at 485M, profiles/r4_b)."""
    if device.type != "cuda":
        return CHUNK_MIN
    free, _ = torch.cuda.mem_get_info(device)
    c = max(CHUNK_MIN, min(CHUNK_MAX, free // 16))
    if total is not None:
        c = max(CHUNK_MIN, min(c, total // 8))
    return int(c) & ~((1 << 20) - 1)


def _eff_end(src) -> int:
    """End of the content that survives Java's trailing-empty-line removal."""
    n = len(src)
    i = n
    while i > 0 and src[i - 1] == 10:
        i -= 1
        if i > 0 and src[i - 1] == 13:
            i -= 1
    return i


class RepeatBuffer:
    """A virtual buffer: ``block`` repeated to ``total`` bytes (synthetic multi-GB streams)."""

    def __init__(self, block: bytes, total: int):
        self.block = block
        self.total = total

    def __len__(self):
        return self.total

    def __getitem__(self, idx):
        if isinstance(idx, int):
            return self.block[idx % len(self.block)]
        start, stop, _ = idx.indices(self.total)
        if start >= stop:
            return b""
        B = len(self.block)
        out = bytearray()
        pos = start
        while pos < stop:
            o = pos % B
            take = min(B - o, stop - pos)
            out += self.block[o:o + take]
            pos += take
        return bytes(out)

    PIN_TILE_BYTES = 256 << 20      # the registered copy holds the block tiled to >= this

    def segments(self, start: int, stop: int):
        """[(offset in ``pinned_block()``, offset from start, length)] covering [start, stop): the
        registered copy is the block tiled (the same byte stream), so a chunk is a few large DMA
        copies instead of one per ~20 MB block."""
        B = len(self.block) * getattr(self, "_reps", 1)
        out, pos = [], start
        while pos < stop:
            b = pos % B
            take = min(B - b, stop - pos)
            out.append((b, pos - start, take))
            pos += take
        return out

    def pinned_block(self) -> Optional[torch.Tensor]:
        """The block as a page-locked CPU tensor (registered once, in place) for direct H2D
        copies, or None when the runtime cannot lock it."""
        if not hasattr(self, "_pin"):
            self._pin = None
            if torch.cuda.is_available() and len(self.block):
                # a private, page-aligned copy (anonymous mapping): the registration covers whole
                # pages of memory this object owns, and is dropped before the mapping
                import mmap
                import weakref
                from ..native import N
                self._reps = max(1, self.PIN_TILE_BYTES // len(self.block))
                B = len(self.block) * self._reps
                self._map = mmap.mmap(-1, B)
                for k in range(self._reps):
                    self._map[k * len(self.block):(k + 1) * len(self.block)] = self.block
                own = np.frombuffer(self._map, dtype=np.uint8)
                if not N.host_register(own.ctypes.data, B):
                    self._reps = 1
                else:
                    self._pin = torch.from_numpy(own)
                    # unregister, then unmap (the finalizer holds the mapping until then)
                    weakref.finalize(self, lambda m, p: N.host_unregister(p), self._map, own.ctypes.data)
        return self._pin

    def copy_into(self, dst: torch.Tensor, start: int, stop: int) -> None:
        """dst[0:stop-start] = self[start:stop] with tensor copies (no Python byte strings)."""
        if not hasattr(self, "_bt"):
            with warnings.catch_warnings():       # read-only source view, only copied from
                warnings.simplefilter("ignore", UserWarning)
                self._bt = torch.from_numpy(np.frombuffer(self.block, dtype=np.uint8))
        B = len(self.block)
        pos, o = start, 0
        while pos < stop:
            b = pos % B
            take = min(B - b, stop - pos)
            dst[o:o + take].copy_(self._bt[b:b + take])
            pos += take
            o += take

    def find(self, sub: bytes, start: int) -> int:
        B = len(self.block)
        pos = start
        while pos < self.total:
            o = pos % B
            j = self.block.find(sub, o)
            if j >= 0 and pos + (j - o) < self.total:
                return pos + (j - o)
            pos += B - o
        return -1

    def rfind(self, sub: bytes, start: int, end: int) -> int:
        B = len(self.block)
        pos = end
        while pos > start:
            o = (pos - 1) % B
            j = self.block.rfind(sub, 0, o + 1)
            if j >= 0:
                r = pos - 1 - (o - j)
                return r if r >= start else -1
            pos -= o + 1
        return -1


@dataclass
class StreamResult:
    total_lines: int
    n_events: int
    summary: dict
    topk_score: np.ndarray
    topk_line: np.ndarray
    topk_pat: np.ndarray
    chunks: int
    bytes: int
    seconds: float
    events: Optional[tuple] = None          # (global line int64, pattern int32, score f64) if kept
    timings: dict = field(default_factory=dict)


class ResidentLog:
    """A log held in HBM for repeated analyses (e.g. re-analysis with a new pattern library): the
    bytes cross PCIe once, as line-aligned chunks with their halos (the same chunk plan as the
    stream), and ``StreamAnalyzer.run(resident)`` then reads them in place -- no host staging, no
    H2D per analysis. Sized for 288 GB of HBM per MI355X: a multi-10-GB log fits with room for
    the analysis workspaces."""

    def __init__(self, chunks: list, nbytes: int, halo: int, chunk_bytes: int):
        self.chunks = chunks            # [(device text (padded), n, lh, rh, end)]
        self.nbytes = nbytes
        self.halo = halo
        self.chunk_bytes = chunk_bytes

    @classmethod
    def load(cls, src, engine: Engine, chunk_bytes: Optional[int] = None) -> "ResidentLog":
        sa = StreamAnalyzer(engine, chunk_bytes=chunk_bytes)
        dev = engine.device
        q: "queue.Queue" = queue.Queue(maxsize=2)
        free_q: Optional[queue.Queue] = None
        if dev.type == "cuda":
            free_q = queue.Queue()
            for _ in range(sa.PINNED_BUFFERS):
                free_q.put((None, None))
        th = threading.Thread(target=sa._producer, args=(src, _eff_end(src), q, 0, free_q), daemon=True)
        th.start()
        chunks, total = [], 0
        while True:
            item = q.get()
            if isinstance(item, BaseException):
                raise item
            if item is None:
                break
            pinned, n, size, lh, rh, end = item
            d = torch.empty(size, dtype=torch.uint8, device=dev)
            d.copy_(pinned[:size], non_blocking=dev.type == "cuda")
            ev = None
            if dev.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
            if free_q is not None:
                free_q.put((pinned, ev))
            chunks.append((d, n, lh, rh, end))
            total += n
        th.join()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return cls(chunks, len(src), engine.lib.halo, sa.chunk_bytes)

    @property
    def device_bytes(self) -> int:
        return sum(c[0].numel() for c in self.chunks)


class StreamAnalyzer:
    def __init__(self, engine: Engine, chunk_bytes: Optional[int] = None, topk: int = 100,
                 keep_events: bool = True):
        """``keep_events=False``: bounded memory for dense matches -- the summary histograms
        accumulate per chunk and only events that can still reach the top-k are kept (exact, see
        ``_prune``), instead of every event's seven factors until the end of the stream."""
        self.engine = engine
        self._auto_chunk = not (chunk_bytes or engine.config["engine.chunk-bytes"])
        self.chunk_bytes = int(chunk_bytes or engine.config["engine.chunk-bytes"] or auto_chunk_bytes(engine.device))
        K._check_k(topk)
        self.topk = topk
        self.keep_events = keep_events
        lib = engine.lib
        off = lib.seq_ev_off
        e0 = np.zeros(max(lib.n_seq_events, 1), np.int64)
        for q in range(off.size - 1):
            e0[off[q]:off[q + 1]] = off[q]
        self.slot_e0 = torch.from_numpy(e0).to(engine.device)

    # ------------------------------------------------------------------ chunk planning
    def _plan(self, src, eff: int, start: int = 0):
        H = self.engine.lib.halo
        pos = start
        k = 0
        while pos < eff or (pos == 0 and eff == 0):
            # ramp-up: chunks double from RAMP_MIN, so the staging -> H2D -> compute pipeline fills
            # in milliseconds instead of one full-size host copy; ramp-down: near the end a chunk is
            # at most RAMP_DOWN of what remains (down to RAMP_MIN), so the drain -- the last chunk's
            # analysis after the last copy -- is a small chunk's, not an 8 GiB one's. Successive
            # ramp-down chunks shrink by 1 - RAMP_DOWN: each chunk's copy must outlast the previous
            # (larger) chunk's analysis, or the copy engine idles (at 1/2 per chunk it did: ~80 ms
            # over a 1B-line stream's tail, profiles/r4_b)
            size = min(self.chunk_bytes, self.RAMP_MIN << min(k, 40))
            rest = eff - pos
            if rest > self.RAMP_END:
                size = min(size, max(self.RAMP_END, int(rest * self.RAMP_DOWN)))
            k += 1
            end = min(eff, pos + size)
            if end < eff:
                j = src.find(b"\n", end - 1)
                end = eff if (j < 0 or j + 1 > eff) else j + 1
            r_end, rh = end, 0
            while rh < H and r_end < eff:
                j = src.find(b"\n", r_end)
                r_end = eff if (j < 0 or j + 1 > eff) else j + 1
                rh += 1
            l_start, lh = pos, 0
            while lh < H and l_start > 0:
                j = src.rfind(b"\n", 0, l_start - 1)
                l_start = 0 if j < 0 else j + 1
                lh += 1
            yield l_start, pos, end, r_end, lh, rh
            if end >= eff:
                break
            pos = end

    PINNED_BUFFERS = 3          # one being filled, one in the H2D copy, one spare
    PRUNE_AT = 1 << 20          # bounded mode: prune the kept events past this many

    def _chrono_bounds(self):
        """[min, max] of the chronological factor over any position (ScoringService.java:123-151:
        piecewise linear through m at 0, 1.5 at e, 1.0 at t, -> 0.5 at the end)."""
        p = self.engine.params
        m, e, t = float(p.max_early_bonus), float(p.early_bonus_threshold), float(p.penalty_threshold)
        # segment endpoints: m (pos 0), 1.5 (pos e), 1.0 (pos t), 1.5 - max(e, t) (late segment
        # start), -> 0.5 (pos 1); m may be configured below 0.5 or above 1.5
        return min(0.5, m), max(m, 1.5, 1.5 - min(e, t, 0.0))

    def _prune(self, ev_gl, ev_pat, ev_fac, cmin: float, cmax: float):
        """Keep only events that can still be in the final top-k. The final score is the
        left-to-right product with the chronological factor of the (not yet known) line count;
        fp64 multiplication is monotone, so evaluating the same product with the factor's min /
        max gives exact lower / upper bounds. Events whose upper bound is below the k-th largest
        lower bound can never enter the top-k (ties keep: the bound test is strict)."""
        gl, pat, fac = torch.cat(ev_gl), torch.cat(ev_pat), torch.cat(ev_fac)
        k = max(1, self.topk)
        if gl.numel() <= k:
            return [gl], [pat], [fac]

        def prod(c):
            v = fac[:, 0] * fac[:, 1]
            v = v * c
            for j in (3, 4, 5):
                v = v * fac[:, j]
            return v * (1.0 - fac[:, 6])
        lb, ub = prod(cmin), prod(cmax)
        thr = torch.topk(lb, k).values[-1]
        keep = ub >= thr
        return [gl[keep]], [pat[keep]], [fac[keep]]
    RAMP_MIN = 64 << 20         # first / last chunk size of the ramps (bytes)
    # ramp-down: a chunk takes at most RAMP_DOWN of what remains, down to RAMP_END. A tail chunk
    # only shortens the drain while its copy outlasts the previous chunk's analysis: s' / copy_rate >=
    # s / analysis_rate + ~5 ms fixed (line count read-back, launches). With a 4k-pattern library
    # (analysis ~68 GB/s vs 57 GB/s PCIe) that allows ~16% shrink per chunk and nothing below ~2 GB
    # (profiles/r4_b: 1/2 per chunk down to 64 MB left 80 ms of copy-engine gaps)
    RAMP_DOWN = 0.16
    RAMP_END = 1 << 30
    PREFETCH = 3                # chunks staged + copied ahead of the one being analysed

    def _producer(self, src, eff, q: "queue.Queue", start: int = 0, free_q: Optional["queue.Queue"] = None,
                  plan=None, direct=None):
        """Stages line-aligned chunks (+ halos) into pinned buffers. On GPU the buffers come from a
        small recycled pool (``free_q``: buffer + the event of the H2D copy that last read it) --
        allocating and pinning a fresh 0.5 GB buffer per chunk costs 30-100 ms, 3x the copy.
        ``plan``: an explicit list of chunks (``_plan`` entries; None = an empty chunk).
        ``direct`` = (device, copy stream, device-buffer pool): a source already in page-locked
        memory (a registered ``RepeatBuffer`` block) is not staged at all -- this thread copies each
        chunk's segments of it straight into a recycled device buffer on the copy stream and hands
        over the device chunk (item tag "dev"). The host only issues copies, the copy engine never
        waits for the analysis thread's syncs, and the stream runs at the PCIe rate (a 3.3 GB
        staged chunk ran at 43 GB/s, profiles/r4_a; copies issued by the analysis thread left
        ~85 ms of gaps in a 1B-line stream's ramp-down, profiles/r4_b)."""
        try:
            if direct is not None and isinstance(src, RepeatBuffer) and src.pinned_block() is not None:
                dev, cs, dev_free = direct
                torch.cuda.set_device(dev)
                blk = src.pinned_block()
                cap = K.padded_len(self.chunk_bytes + (self.chunk_bytes >> 4))
                for ent in (plan if plan is not None else self._plan(src, eff, start)):
                    l_start, pos, end, r_end, lh, rh = ent
                    n = r_end - l_start
                    size = K.padded_len(n)
                    buf, used = dev_free.get()
                    if used is not None:
                        used.synchronize()              # the analysis that read it has run
                    with torch.cuda.stream(cs):
                        if buf is None or buf.numel() < size:
                            buf = None
                            buf = torch.empty(max(size, cap), dtype=torch.uint8, device=dev)
                        d = buf[:size]
                        for b, o, take in src.segments(l_start, r_end):
                            d[o:o + take].copy_(blk[b:b + take], non_blocking=True)
                        d[n:size].zero_()
                        ev = torch.cuda.Event()
                        ev.record(cs)
                    q.put(("dev", buf, d, n, lh, rh, end, ev))
                q.put(None)
                return
            flat = None
            if not isinstance(src, RepeatBuffer):
                # zero-copy view of bytes / bytearray / memoryview / mmap; only ever read (copied
                # into the pinned stage), so torch's warning about read-only sources does not apply
                if len(src):
                    with warnings.catch_warnings():
                        warnings.simplefilter("ignore", UserWarning)
                        flat = torch.from_numpy(np.frombuffer(src, dtype=np.uint8))
            for ent in (plan if plan is not None else self._plan(src, eff, start)):
                if ent is None:                               # no chunk for this rank in this step
                    q.put((torch.zeros(K.padded_len(0), dtype=torch.uint8), 0, K.padded_len(0), 0, 0, -1))
                    continue
                l_start, pos, end, r_end, lh, rh = ent
                n = r_end - l_start
                size = K.padded_len(n)
                if free_q is not None:
                    pinned, ev = free_q.get()
                    if ev is not None:
                        ev.synchronize()                      # its previous H2D copy is done
                    if pinned is None or pinned.numel() < size:
                        cap = max(size, K.padded_len(self.chunk_bytes + (self.chunk_bytes >> 4)))
                        pinned = None
                        pinned = registered_empty(cap)      # SDMA-copied pages (utils/hostmem.py)
                else:
                    pinned = torch.empty(size, dtype=torch.uint8)
                if n:
                    if flat is not None:
                        pinned[:n].copy_(flat[l_start:r_end])       # one (multi-threaded) copy
                    else:
                        src.copy_into(pinned, l_start, r_end)
                pinned[n:size].zero_()
                q.put((pinned, n, size, lh, rh, end))
            q.put(None)
        except BaseException as e:  # noqa: BLE001
            q.put(e)

    # ------------------------------------------------------------------ run
    def run(self, src, on_chunk: Optional[Callable] = None, checkpoint: Optional[str] = None,
            checkpoint_every: int = 1, resume: Optional[str] = None,
            fail_after_chunks: Optional[int] = None) -> StreamResult:
        """Analyse ``src`` (bytes-like, mmap or RepeatBuffer).

        checkpoint / checkpoint_every: after every N chunks write the stream cursor and all carries
        (global line offset, running frequency counts, sequence-chain state, the frequency carry
        the stream started with, events so far) to an ``.npz``; ``resume`` continues from it and
        produces exactly the uninterrupted result. ``fail_after_chunks`` injects a
        failure (tests)."""
        t0 = time.perf_counter()
        eng = self.engine
        lib = eng.lib
        dev = eng.device
        eff = src.nbytes if isinstance(src, ResidentLog) else _eff_end(src)
        if not isinstance(src, ResidentLog) and eff == 0 and len(src) > 0 and src.find(b"\n", 0) >= 0:
            empty = {"significantEvents": 0, "highestSeverity": "NONE", "severityDistribution": {}}
            z = np.zeros(0)
            return StreamResult(0, 0, empty, z, z.astype(np.int64), z.astype(np.int64), 0, len(src), 0.0)
        nkeys = len(lib.freq_ids)
        resident = isinstance(src, ResidentLog)
        if self._auto_chunk and not resident:
            self.chunk_bytes = auto_chunk_bytes(dev, eff)       # (same on resume: eff is the whole stream)
        if resident and src.halo < lib.halo:
            raise ValueError(f"resident log staged with {src.halo} halo lines, the library needs {lib.halo}")
        start = 0
        P, S = len(lib.patterns), len(lib.sev_names)
        hist = torch.zeros(P + S + 1, dtype=torch.int64, device=dev)      # bounded mode: running histograms
        n_events = 0
        first_pat = None
        cmin, cmax = self._chrono_bounds()
        if resume:
            with np.load(resume, allow_pickle=False) as ck:
                start = int(ck["pos"])
                line_base = int(ck["line_base"])
                chunks = int(ck["chunks"])
                nbytes_total = int(ck["nbytes"])
                freq_carry = torch.from_numpy(ck["freq_carry"]).to(dev)
                run_counts = torch.from_numpy(ck["run_counts"]).to(dev)
                seq_state = torch.from_numpy(ck["seq_state"]).to(dev)
                ev_gl = [torch.from_numpy(ck["gl"]).to(dev)]
                ev_pat = [torch.from_numpy(ck["pat"]).to(dev)]
                ev_fac = [torch.from_numpy(ck["fac"]).to(dev)]
        else:
            freq_carry = eng.freq_carry()
            run_counts = torch.zeros(max(nkeys, 1), dtype=torch.int64, device=dev)
            seq_state = torch.zeros(max(lib.n_seq_events, 1), dtype=torch.uint8, device=dev)
            line_base = 0
            ev_gl, ev_pat, ev_fac = [], [], []
            chunks = 0
            nbytes_total = 0
        q: "queue.Queue" = queue.Queue(maxsize=2)
        free_q: Optional[queue.Queue] = None
        dev_free: Optional[queue.Queue] = None
        if dev.type == "cuda" and not resident:
            free_q = queue.Queue()
            for _ in range(self.PINNED_BUFFERS):
                free_q.put((None, None))
            dev_free = queue.Queue()
            for _ in range(self.PREFETCH + 1):
                dev_free.put((None, None))
        copy_stream = torch.cuda.Stream(dev) if dev.type == "cuda" and not resident else None
        # the backtracker side path reads the chunk's pinned host bytes: their buffer is recycled
        # only after this chunk's prepare (and such chunks are staged, not copied directly)
        hold = bool(lib.host_plan)
        th = None
        if resident:
            if resume:
                raise ValueError("resume applies to host streams, not resident logs")
            res_iter = iter(src.chunks)
        else:
            direct = (dev, copy_stream, dev_free) if dev.type == "cuda" and not hold else None
            th = threading.Thread(target=self._producer, args=(src, eff, q, start, free_q),
                                  kwargs={"direct": direct}, daemon=True)
            th.start()

        def save(pos_next):
            def cat(xs, dt, shape):
                return torch.cat(xs).cpu().numpy() if xs else np.zeros(shape, dt)
            tmp = checkpoint + ".tmp"
            with open(tmp, "wb") as f:
                np.savez(f, pos=pos_next, line_base=line_base, chunks=chunks, nbytes=nbytes_total,
                         freq_carry=freq_carry.cpu().numpy(), run_counts=run_counts.cpu().numpy(),
                         seq_state=seq_state.cpu().numpy(), gl=cat(ev_gl, np.int64, (0,)),
                         pat=cat(ev_pat, np.int32, (0,)), fac=cat(ev_fac, np.float64, (0, 7)))
            import os
            os.replace(tmp, checkpoint)

        def fetch():
            if resident:                        # already in HBM: nothing to stage or copy
                c = next(res_iter, None)
                return None if c is None else (c[0], c[1], c[2], c[3], None, c[4], None)
            item = q.get()
            if isinstance(item, BaseException):
                raise item
            if item is None:
                return None
            if item[0] == "dev":                # copied by the producer into a pooled device buffer
                _, buf, d, n, lh, rh, end, ev = item
                return d, n, lh, rh, ev, end, buf
            pinned, n, size, lh, rh, end = item
            if copy_stream is not None:
                with torch.cuda.stream(copy_stream):
                    d = torch.empty(size, dtype=torch.uint8, device=dev)
                    d.copy_(pinned[:size], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                if not hold:
                    free_q.put((pinned, ev))                   # recycled once the copy is done
                return d, n, lh, rh, ev, end, pinned
            return pinned, n, lh, rh, None, end, pinned

        # copies run PREFETCH chunks ahead of the analysis: with one chunk ahead, a copy shorter than
        # the previous chunk's analysis (the ramp-down) left the copy engine idle until the next
        # iteration issued the following one
        ahead: "deque" = deque()
        ended = False

        # hold mode keeps every staged chunk's pinned buffer until its prepare: the consumer then holds
        # the current chunk + the look-ahead, so the look-ahead must leave the producer one buffer of
        # the pool to fill, or refill() waits on a chunk the producer cannot stage
        depth = min(self.PREFETCH, self.PINNED_BUFFERS - 1) if hold and free_q is not None else self.PREFETCH

        def refill():
            nonlocal ended
            while not ended and len(ahead) < depth:
                it = fetch()
                if it is None:
                    ended = True
                else:
                    ahead.append(it)

        refill()
        while ahead:
            text, n, lh, rh, ev, chunk_end, host = ahead.popleft()
            dev_buf = None
            if host is not None and host.is_cuda:       # a pooled device buffer (direct copies)
                dev_buf, host = host, None
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
                text.record_stream(torch.cuda.current_stream(dev))
            refill()                           # stage + copy the next chunks meanwhile
            ls, ll = K.split_chunk_lines(text, n)
            L = ls.numel()
            own_lo, own_hi = lh, L - rh
            segs = Segments.scalar(0, L, own_lo, own_hi, line_base - own_lo, 1 << 62, dev)
            prep = eng.prepare(text, n, ls, ll, segs, host_text=host[:n].numpy() if hold and host is not None else None,
                               split_trim=False)
            if hold and free_q is not None and host is not None:
                free_q.put((host, ev))
            chain = eng.seq_chain_table(prep, own_lo, own_hi)
            res = eng.finish(prep, segs, freq_carry + run_counts, seq_state, with_factors=True)
            if dev_buf is not None:            # every kernel reading the chunk is queued: recycle
                used = torch.cuda.Event()
                used.record(torch.cuda.current_stream(dev))
                dev_free.put((dev_buf, used))
            if lib.n_seq_events:
                k = chain.to(torch.int64)
                prev = seq_state[(self.slot_e0 + k.clamp(min=0))]
                seq_state = torch.where(k < 0, torch.ones_like(seq_state), prev)
            run_counts = run_counts + prep.freq_counts[:max(nkeys, 1)]
            if res.ev_line.numel():
                gl_c = res.ev_line.to(torch.int64) - own_lo + line_base
                if self.keep_events:
                    ev_gl.append(gl_c)
                    ev_pat.append(res.ev_pat)
                    ev_fac.append(res.factors)
                else:
                    # bounded: histograms now, and only events that may still make the top-k
                    K.summarize(res.score, res.ev_pat, res.ev_line, 1, eng.tabs["sev_index"], P, S, ws=eng.ws,
                                hist_out=hist)
                    n_events += int(res.ev_line.numel())
                    if first_pat is None:
                        first_pat = int(res.ev_pat[0].item())
                    ev_gl.append(gl_c)
                    ev_pat.append(res.ev_pat)
                    ev_fac.append(res.factors)
                    if sum(x.numel() for x in ev_gl) > self.PRUNE_AT:
                        ev_gl, ev_pat, ev_fac = self._prune(ev_gl, ev_pat, ev_fac, cmin, cmax)
            if on_chunk is not None:
                on_chunk(chunks, line_base, own_hi - own_lo)
            line_base += own_hi - own_lo
            nbytes_total += n
            chunks += 1
            if checkpoint and chunks % max(1, checkpoint_every) == 0:
                save(chunk_end)
            if fail_after_chunks is not None and chunks >= fail_after_chunks:
                raise RuntimeError("injected stream failure after chunk %d" % chunks)
        if th is not None:
            th.join()
        N = max(line_base, 1)
        if ev_gl:
            gl = torch.cat(ev_gl)
            pat = torch.cat(ev_pat)
            fac = torch.cat(ev_fac)
            # reference product order with the true chronological factor (k_rescore)
            score = K.rescore(gl, fac, N, eng.sp_tuple)
        else:
            gl = torch.zeros(0, dtype=torch.int64, device=dev)
            pat = torch.zeros(0, dtype=torch.int32, device=dev)
            score = torch.zeros(0, dtype=torch.float64, device=dev)
        eng.commit_frequency(run_counts[:nkeys])
        # summary + top-k in one kernel chain (summarize.hip): severity histogram, k best rows
        rows, _, sc, _ = K.summarize(score, pat, gl, max(1, self.topk), eng.tabs["sev_index"], P, S, ws=eng.ws)
        if self.keep_events:
            n_events = int(score.numel())
            first = int(pat[0].item()) if pat.numel() else None
        else:
            sc = hist[P:P + S]
            first = first_pat
        k = min(self.topk, n_events)
        top = rows[:k].cpu().numpy()
        summary = eng.summary_from_severity(sc.cpu().numpy(), first)
        out = StreamResult(line_base, n_events, summary, top[:, 0].copy(), top[:, 1].astype(np.int64),
                           top[:, 2].astype(np.int64), chunks, nbytes_total, time.perf_counter() - t0)
        if self.keep_events:
            out.events = (gl.cpu().numpy(), pat.cpu().numpy(), score.cpu().numpy())
        return out


class ShardedStreamAnalyzer:
    """One long log streamed over the ranks of a process group (one process per GPU): the chunk
    plan of ``StreamAnalyzer`` is cut into steps of ``world`` consecutive chunks, rank r analyses
    chunk r of every step, and each step is a data-parallel step (``ShardedAnalyzer.step``) whose
    carries come from the earlier steps (``StreamCarry``) -- the SAME carry protocol for chunks and
    for ranks: frequency counts of everything before (window totals + earlier steps
    + earlier ranks of the step), the composed backward sequence-chain state, the global line
    offset; N stays open and every event keeps its factors, rescored at the end with the true N
    (the reference's left-to-right product, ``k_rescore``). Every rank stages only its own chunks
    (reading its byte ranges of the shared source), so a 1B-line log costs each of 8 GPUs 1/8 of
    the PCIe ingest. The summary and top-k are merged across ranks at the end (one all-gather);
    every rank returns the same ``StreamResult``, with ``events`` = its own events."""

    def __init__(self, engine: Engine, chunk_bytes: Optional[int] = None, topk: int = 100, group=None):
        from .dp import ShardedAnalyzer
        self.engine = engine
        self.group = group
        self.sa = StreamAnalyzer(engine, chunk_bytes=chunk_bytes, topk=topk, keep_events=True)
        self.dp = ShardedAnalyzer(engine, group)
        self.topk = topk

    def run(self, src) -> StreamResult:
        from .dp import StreamCarry, all_gather_inplace, world
        t0 = time.perf_counter()
        eng = self.engine
        lib = eng.lib
        dev = eng.device
        rank, W = world()
        eff = _eff_end(src)
        if eff == 0 and len(src) > 0 and src.find(b"\n", 0) >= 0:
            empty = {"significantEvents": 0, "highestSeverity": "NONE", "severityDistribution": {}}
            z = np.zeros(0)
            return StreamResult(0, 0, empty, z, z.astype(np.int64), z.astype(np.int64), 0, len(src), 0.0)
        if self.sa._auto_chunk:
            self.sa.chunk_bytes = auto_chunk_bytes(dev, max(eff // W, 1))
        plan = list(self.sa._plan(src, eff))                      # the same plan on every rank
        steps = (len(plan) + W - 1) // W
        mine = [plan[s * W + rank] if s * W + rank < len(plan) else None for s in range(steps)]
        nkeys, ns = len(lib.freq_ids), max(lib.n_seq_events, 1)
        carry = StreamCarry(eng.freq_carry()[:max(nkeys, 1)].clone() if nkeys else
                            torch.zeros(1, dtype=torch.int64, device=dev),
                            torch.zeros(ns, dtype=torch.uint8, device=dev), 0)
        start_carry = carry.freq.clone()
        q: "queue.Queue" = queue.Queue(maxsize=2)
        free_q: Optional[queue.Queue] = None
        if dev.type == "cuda":
            free_q = queue.Queue()
            for _ in range(self.sa.PINNED_BUFFERS):
                free_q.put((None, None))
        th = threading.Thread(target=self.sa._producer, args=(src, eff, q, 0, free_q, mine), daemon=True)
        th.start()
        copy_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        hold = bool(lib.host_plan)             # backtracker side path: reads the pinned host bytes
        ev_gl, ev_pat, ev_fac = [], [], []
        nbytes_total = 0
        for _ in range(steps):
            item = q.get()
            if isinstance(item, BaseException):
                raise item
            pinned, n, size, lh, rh, _end = item
            idle = _end < 0                                      # own no line this step: a placeholder
            recycle = copy_stream is not None and not idle       # (not from the pinned pool)
            host_text = None
            if copy_stream is not None:
                with torch.cuda.stream(copy_stream):
                    text = torch.empty(size, dtype=torch.uint8, device=dev)
                    text.copy_(pinned[:size], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                torch.cuda.current_stream(dev).wait_event(ev)
                text.record_stream(torch.cuda.current_stream(dev))
                if hold and not idle:
                    host_text = pinned[:n].numpy()              # the side path reads the pinned bytes
                elif recycle:
                    free_q.put((pinned, ev))
                    recycle = False
            else:
                text = pinned
            if idle:
                ls = torch.zeros(0, dtype=torch.int64, device=dev)
                ll = torch.zeros(0, dtype=torch.int32, device=dev)
            else:
                ls, ll = K.split_chunk_lines(text, n)
            out = self.dp.step(text, n, ls, ll, lh, rh, topk=0, stream_carry=carry, split_trim=False,
                               host_text=host_text)
            if recycle:                                          # hold mode: after the side path's read
                free_q.put((pinned, ev))
            res = out.result
            if res.ev_line.numel():
                ev_gl.append(res.ev_line.to(torch.int64) - out.own_lo + out.own_start_dev)
                ev_pat.append(res.ev_pat)
                ev_fac.append(res.factors)
            carry = StreamCarry(carry.freq + out.freq_counts[:carry.freq.numel()] if nkeys else carry.freq,
                                out.seq_next, carry.line_base + out.total_lines)
            nbytes_total += n
        th.join()
        N_total = max(carry.line_base, 1)
        if ev_gl:
            gl, pat, fac = torch.cat(ev_gl), torch.cat(ev_pat), torch.cat(ev_fac)
            score = K.rescore(gl, fac, N_total, eng.sp_tuple)
        else:
            gl = torch.zeros(0, dtype=torch.int64, device=dev)
            pat = torch.zeros(0, dtype=torch.int32, device=dev)
            score = torch.zeros(0, dtype=torch.float64, device=dev)
        if nkeys:
            eng.commit_frequency(carry.freq - start_carry)        # every rank: the stream's global counts
        # merge: [pattern hist | severity hist | first event (line, pattern) | top-k rows] per rank
        P, S = len(lib.patterns), len(lib.sev_names)
        k = max(1, self.topk)
        H = P + S
        red2 = torch.empty((W, H + 2 + 3 * k), dtype=torch.int64, device=dev)
        row = red2[rank]
        row[:H].zero_()
        row[H] = int(gl[0].item()) if gl.numel() else (1 << 62)
        row[H + 1] = int(pat[0].item()) if pat.numel() else -1
        K.summarize(score, pat, gl, k, eng.tabs["sev_index"], P, S, ws=eng.ws, hist_out=row[:H],
                    rows_out=row[H + 2:].view(torch.float64).view(k, 3))
        all_gather_inplace(red2, self.group)
        hist = red2[:, :H].sum(0)
        rows = red2[:, H + 2:].contiguous().view(torch.float64).view(-1, 3)
        top = (K.topk_rows(rows, k, ws=eng.ws) if rows.shape[0] > k else rows).cpu().numpy()
        n_events = int(hist[:P].sum().item())
        firsts = red2[:, H:H + 2].cpu().numpy()
        first = None
        if n_events:
            j = int(np.lexsort((firsts[:, 1], firsts[:, 0]))[0])
            first = int(firsts[j, 1])
        kk = min(self.topk, n_events)
        summary = eng.summary_from_severity(hist[P:P + S].cpu().numpy(), first)
        out = StreamResult(carry.line_base, n_events, summary, top[:kk, 0].copy(), top[:kk, 1].astype(np.int64),
                           top[:kk, 2].astype(np.int64), len(plan), nbytes_total, time.perf_counter() - t0)
        out.events = (gl.cpu().numpy(), pat.cpu().numpy(), score.cpu().numpy())
        return out
