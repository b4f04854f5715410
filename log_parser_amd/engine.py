"""Device pipeline orchestration: bytes -> line index -> match -> events -> scores -> summary.

Reference call stack being replaced: ``Parse.parseLogs`` ->
``AnalysisService.analyze`` (split, per-request compile, line x set x pattern ``find()``,
context, ``ScoringService.calculateScore`` per hit) -> ``buildMetadata`` / ``buildSummary``.

Here one request (or a batch of requests, or one rank's shard of a huge log) is a
*segmented line batch* resident in device memory:

  text (uint8, padded)  line_start[L] int64  line_len[L] int32
  segments: per document / shard  lo, hi (available local lines), own_lo, own_hi (lines that
            emit events), g0 (global index of local line lo), n (document line count N)

and every stage is a bulk kernel over the whole batch:

  1. k_prefilter / k_pf_verify   literal bloom + hash filter -> (regex, line) candidates
  2. post-match pipeline         (csrc/kernels/lp_post.hip) sort + dedupe + DFA verify ->
                                 CSR per regex (shared by primary, secondary, sequence roles),
                                 events in (line, pattern) order on owned lines, in-batch
                                 frequency ranks, context features of window lines only
  3. k_score                     fused fp64 7-factor score, one lane per event, frequency carry fused
  4. summary                     severity histogram / highest severity / top-k

``prepare`` (1-2) needs no global information; ``finish`` (3) takes the line count N, the
frequency carry and the sequence-chain carry, which the data-parallel, streaming and
multi-engine serving drivers produce in between.
"""
from __future__ import annotations

import logging
import os
import threading
import time
import uuid
import warnings
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .frequency import DeviceFrequencyState, FrequencyState
from .golden import SEVERITY_ORDER
from .models.compiled import CompiledLibrary
from .native import N, host_thread_budget
from .ops import kernels as K
from .utils import tracing as TR
from .utils.config import Config, ScoringParams

log = logging.getLogger("log_parser_amd.engine")


def resolve_device(spec: str = "auto") -> torch.device:
    if spec == "auto":
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(spec)


@dataclass
class Segments:
    lo: torch.Tensor
    hi: torch.Tensor
    own_lo: torch.Tensor
    own_hi: torch.Tensor
    g0: torch.Tensor
    n: torch.Tensor

    @staticmethod
    def scalar(lo: int, hi: int, own_lo: int, own_hi: int, g0: int, n: int, device, upload=None) -> "Segments":
        """One segment (two small host->device copies instead of six; with an engine's
        ``upload``, one async copy through its pinned buffer)."""
        if upload is not None:
            t32, t64 = upload([np.array([lo, hi, own_lo, own_hi], np.int32), np.array([g0, n], np.int64)])
        else:
            t32 = torch.tensor([lo, hi, own_lo, own_hi], dtype=torch.int32, device=device)
            t64 = torch.tensor([g0, n], dtype=torch.int64, device=device)
        return Segments(t32[0:1], t32[1:2], t32[2:3], t32[3:4], t64[0:1], t64[1:2])

    @staticmethod
    def single(L: int, device) -> "Segments":
        return Segments.scalar(0, L, 0, L, 0, L, device)

    @staticmethod
    def doc_arrays(doc_line_off: np.ndarray):
        """Host arrays (lo, hi, g0, n) of a batch of whole documents (every line owned)."""
        lo = doc_line_off[:-1].astype(np.int32)
        hi = doc_line_off[1:].astype(np.int32)
        n = (doc_line_off[1:] - doc_line_off[:-1]).astype(np.int64)
        return lo, hi, np.zeros_like(n), n

    @staticmethod
    def from_doc_offsets(doc_line_off: np.ndarray, device) -> "Segments":
        lo, hi, g0, n = (torch.from_numpy(a).to(device) for a in Segments.doc_arrays(doc_line_off))
        return Segments(lo, hi, lo, hi, g0, n)

    def seg_and_owned(self, lines: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Segment id and ownership of the given line ids (only hit lines, never all L lines)."""
        if self.lo.numel() == 1:
            seg = torch.zeros_like(lines)
        else:
            seg = (torch.searchsorted(self.lo, lines, right=True).to(torch.int32) - 1).clamp(min=0)
        owned = (lines >= self.own_lo[seg.long()]) & (lines < self.own_hi[seg.long()])
        return seg, owned


@dataclass
class Prepared:
    ev_line: torch.Tensor
    ev_pat: torch.Tensor
    ev_seg: torch.Tensor
    ev_rank: torch.Tensor               # rank among earlier in-batch events of the same freq key
    ev_fkey: torch.Tensor               # freq key per event (-1: none)
    freq_counts: torch.Tensor
    hits: torch.Tensor
    hit_off: torch.Tensor
    hit_line: torch.Tensor
    feat: torch.Tensor
    n_lines: int
    timings: Dict[str, float] = field(default_factory=dict)
    out_buf: Optional[torch.Tensor] = None   # K.results_buffer holding line / pattern / segment / counts
    # deferred counts (``prepare(defer=True)``): the arrays above are capacities; cnt = device
    # [gram hits, candidates, verified hits, unique hits, events, events that fit (0 on overflow)],
    # caps = their host capacities
    cnt: Optional[torch.Tensor] = None
    caps: Optional[Dict[str, int]] = None

    @property
    def ne_dev(self) -> Optional[torch.Tensor]:
        """The device event count later kernels read: 0 when the events overflowed their buffer."""
        return None if self.cnt is None else self.cnt[5:6]


@dataclass
class RunResult:
    """Device-resident output of one pipeline run (events in reference order)."""
    ev_line: torch.Tensor
    ev_pat: torch.Tensor
    ev_seg: torch.Tensor
    score: torch.Tensor
    factors: Optional[torch.Tensor]
    freq_counts: torch.Tensor           # per freq key, matches in this run
    hit_keys: torch.Tensor              # sorted unique (regex<<32 | line)
    hit_off: torch.Tensor
    n_lines: int
    timings: Dict[str, float] = field(default_factory=dict)
    out_buf: Optional[torch.Tensor] = None   # K.results_buffer: every host-bound result, one D2H


def summary_from_severity(lib, sev_hist: np.ndarray, first_pat: Optional[int]) -> dict:
    """AnalysisSummary (AnalysisService.java:188-215) from the summary kernel's histogram over the
    library's distinct severity names: the highest known severity wins; with none known, the
    severity of the first event in reference order (the reference's first strict improvement)."""
    dist = {lib.sev_names[s]: int(sev_hist[s]) for s in np.nonzero(sev_hist)[0]}
    n = sum(dist.values())
    if n == 0:
        return {"significantEvents": 0, "highestSeverity": "NONE", "severityDistribution": {}}
    best_idx, best = -1, None
    for s in dist:
        if s in SEVERITY_ORDER and SEVERITY_ORDER.index(s) > best_idx:
            best_idx, best = SEVERITY_ORDER.index(s), s
    if best is None and first_pat is not None:
        best = lib.severity[first_pat]
    return {"significantEvents": n, "highestSeverity": best, "severityDistribution": dist}


def _ro_view(data) -> torch.Tensor:
    """uint8 tensor view of a bytes-like object without copying (never written through)."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")            # "non-writable buffer" -- we only read it
        return torch.from_numpy(np.frombuffer(data, dtype=np.uint8))


class FrequencyTurn:
    """Arrival-order gate for the frequency state when several engines (GPUs) analyse batches
    concurrently: batch `seq` reads the persistent carry and records its counts only after every
    earlier batch recorded theirs (penalty before record, ScoringService.java:84-88, in request
    arrival order). Matching, events and context features run before the gate, concurrently;
    only the fused score kernel + the counts read-back are serialised."""

    def __init__(self):
        self._cv = threading.Condition()
        self._next = 0
        self._done: set = set()

    def wait(self, seq: int) -> None:
        with self._cv:
            while self._next < seq:
                self._cv.wait()

    def done(self, seq: int) -> None:
        """Idempotent; may be called out of order (a failed batch releases its slot)."""
        with self._cv:
            if seq < self._next:
                return
            self._done.add(seq)
            while self._next in self._done:
                self._done.discard(self._next)
                self._next += 1
            self._cv.notify_all()


class SharedWindowTurn:
    """Arrival order for several engines sharing ONE device-resident frequency window (GPUs of
    a node reading / recording it over xGMI peer access, or streams of one GPU): ``host`` orders the
    ring's host bookkeeping (record timestamps, tail bound), ``dev`` (``N.WindowTurn``, also used
    inside the native request runner with the GIL released) orders the window sections on the
    device -- eviction, score with the carry, record. Matching runs before both, concurrently."""

    def __init__(self):
        self.host = FrequencyTurn()
        self.dev = N.WindowTurn()

    def wait(self, seq: int) -> None:
        self.host.wait(seq)
        self.dev.wait(seq)

    def done(self, seq: int) -> None:
        self.host.done(seq)
        self.dev.done(seq)


class ProcessWindowTurn(SharedWindowTurn):
    """The same two turns across the serving PROCESSES of a node (``serve/procs.py``): both live
    in the shared segment (``N.ProcShared``: ``host`` / ``dev`` are ``N.ProcTurn``) and a batch's
    sequence number is its arrival ticket there (``take``). The ticket is drawn LATE: by the native
    request runner once the batch's matching has finished on its GPU (``RequestRunner.run(hw=)``),
    by the Python paths right before their window section -- never when the batch enters its
    device stage, so no process waits on another's matching."""

    def __init__(self, shared):
        self.shared = shared
        self.host = shared.host
        self.dev = shared.dev

    def take(self) -> int:
        return self.shared.take()


@dataclass
class BatchJob:
    """One continuous batch between the pipeline stages (pack -> device -> emit)."""
    logs: Sequence
    t0: float
    tm: Optional[dict] = None
    number: int = 0                     # batch number of the engine (fault injection)
    whole: bool = False                 # one huge document, analysed by analyze_json
    stage: Optional[Stage] = None       # staging buffers from the engine's StagePool
    staged: Optional[tuple] = None      # (host view, line_start, line_len, doc_line_off, nbytes)
    n_lines: int = -1                   # >= 0: the line index is in stage.idx (pinned)
    ev: Optional[tuple] = None          # (ev_line, ev_pat, ev_seg, score, freq counts) on the host
    timings: Optional[dict] = None
    outs: Optional[List[bytes]] = None  # responses computed by the device stage itself
    recorded: bool = False              # its counts entered the frequency window (a fallback must not re-record)
    pre_token: int = 0                  # RequestRunner.prefetch_text token (its text already uploading)


class Stage:
    """One batch's (pinned) host staging: packed request bytes + the line index the packer writes
    straight into ``idx`` (int64 starts for ``cap`` lines, then int32 lengths), so both reach the
    device with plain async copies and no intermediate host copy."""

    def __init__(self, pinned: bool, nbytes: int, nlines: int):
        self.pinned = pinned
        self.buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=pinned)
        self.want = 0                       # bytes the request runner's single-copy upload wants
        self.own_buf: Optional[torch.Tensor] = None   # buf while a request's pinned buffer stands in
        self.cap = 0
        self.idx: Optional[torch.Tensor] = None
        self.grow_idx(nlines)

    def grow_buf(self, nbytes: int) -> None:
        self.buf = None
        self.buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=self.pinned)

    def grow_idx(self, nlines: int) -> None:
        self.idx = None
        self.cap = int(nlines)
        self.idx = torch.empty(12 * self.cap, dtype=torch.uint8, pin_memory=self.pinned)

    def starts(self, n: int) -> torch.Tensor:
        return self.idx[:8 * n].view(torch.int64)

    def lens(self, n: int) -> torch.Tensor:
        return self.idx[8 * self.cap:8 * self.cap + 4 * n].view(torch.int32)


class StagePool:
    """Recycled ``Stage`` buffers, one per batch in flight. ``take`` blocks when ``limit`` stages
    are out: the back-pressure of the serving pipeline. ``prewarm`` sizes every stage for a batch
    of ``nbytes`` up front (a server, before it accepts: no pinned allocation on a request's path)."""

    def prewarm(self, nbytes: int, nlines: int) -> None:
        with self._cv:
            free = list(self._free)
            self._free.clear()
        stages = []
        for st in free:
            if st.buf is not None and st.buf.numel() < nbytes:
                st.grow_buf(nbytes)
            if st.idx is not None and st.cap < nlines:
                st.grow_idx(nlines)
            stages.append(st)
        while len(stages) < self.limit:
            stages.append(Stage(self.pinned, nbytes, nlines))
        with self._cv:
            self._free.extend(stages)
            self._cv.notify_all()

    def __init__(self, pinned: bool, initial: int, limit: int = 3):
        self.pinned, self.initial, self.limit = pinned, initial, limit
        self._free: List[Stage] = []
        self._out = 0
        self._cv = threading.Condition()

    def take(self) -> Stage:
        with self._cv:
            while not self._free and self._out >= self.limit:
                self._cv.wait()
            self._out += 1
            while self._free:
                st = self._free.pop()
                if st.buf is not None and st.idx is not None:   # (a failed grow leaves None)
                    return st
        try:
            return Stage(self.pinned, self.initial, self.initial // 16)
        except BaseException:               # e.g. pinned allocation failed: give the slot back
            with self._cv:
                self._out -= 1
                self._cv.notify()
            raise

    def give(self, st: Stage) -> None:
        with self._cv:
            self._out -= 1
            self._free.append(st)
            self._cv.notify()


class Engine:
    def __init__(self, library: CompiledLibrary, config: Optional[Config] = None,
                 device: Optional[torch.device] = None, freq: Optional[FrequencyState] = None):
        self.config = config or Config.load()
        self.lib = library
        self.params: ScoringParams = library.params
        self.device = device if device is not None else resolve_device(self.config["engine.device"])
        if freq is None:
            # one engine owning a GPU keeps the sliding window in HBM (no per-batch H2D / D2H);
            # CPU engines and engines sharing one state across GPUs use the host state
            if self.device.type == "cuda" and bool(self.config.get("engine.frequency.device-resident", True)):
                freq = DeviceFrequencyState(library.freq_ids, self.params.freq_window_hours, self.device)
            else:
                freq = FrequencyState(self.params.freq_window_hours)
        self.freq = freq
        self.cand_cap = int(self.config["engine.candidate-capacity"])
        # per-stage HIP-event timers (utils/tracing.py); engine.trace also reports them per response
        self.trace = bool(self.config.get("engine.trace", False))
        self.profile = self.trace
        # context features: "mfma" = NFA state-transition GEMM (k_nfa_mfma), "dfa" = 4 byte DFAs (k_feat)
        self.context_engine = str(self.config["engine.context-engine"])
        self.log_matches = bool(self.config["server.log-matches"])
        self.fault_every = int(self.config["engine.fault-inject-every"])   # tests: injected device faults
        self.fault_after_record = int(self.config.get("engine.fault-inject-after-record", 0))
        self._batches = 0
        self.tabs = library.device_tables(self.device)
        self.ws = K.Workspace(self.device)          # post-match pipeline scratch (grow-only)
        self.arena = K.MatchArena()                 # matcher output capacities (GPU, adaptive)
        self.upload = K.Uploader(self.device)       # batch line index / segments / carry: one H2D
        self.sp_tuple = self.score_param_tuple(self.params)
        self._pinned: Optional[torch.Tensor] = None
        # batch staging buffers (pinned on GPU), recycled; one per batch in flight in the pipeline
        self._stage_pool = StagePool(pinned=self.device.type == "cuda", initial=K.padded_len(1 << 20))
        # second compute stream: literal-free scans overlap the prefilter chain (K.match_and_hits)
        self._side = None
        self._pf_stream = None
        self._doc_segs = None                       # run_document: (L, Segments) of the last document
        self._host_side = None                      # ops.side_path.HostSide (device-fed backtracker regexes)
        self._runner = None                         # N.RequestRunner (built on first use) / False
        if self.device.type == "cuda":
            props = torch.cuda.get_device_properties(self.device)
            self.n_cus = int(props.multi_processor_count)
            self.pf_grid = self.n_cus * 4
            if bool(self.config.get("engine.scan-stream", True)):
                self._side = (torch.cuda.Stream(self.device), torch.cuda.Event(), torch.cuda.Event())
            # the early literal prefilter's own stream (prefilter_early)
            if bool(self.config.get("engine.prefilter-stream", True)):
                self._pf_stream = torch.cuda.Stream(self.device)
        else:
            self.n_cus = 1
            self.pf_grid = 1

    # ------------------------------------------------------------------ staging
    def stage_text(self, data: bytes) -> Tuple[torch.Tensor, int]:
        """Copy request bytes into a padded device buffer (pinned staging + async H2D)."""
        n = len(data)
        size = K.padded_len(n)
        # read-only zero-copy view of the request bytes; copied once (multi-threaded) into staging
        src = _ro_view(data) if n else torch.empty(0, dtype=torch.uint8)
        if self.device.type == "cuda":
            if self._pinned is None or self._pinned.numel() < size:
                self._pinned = torch.empty(max(size, 1 << 20), dtype=torch.uint8, pin_memory=True)
            self._pinned[:n].copy_(src)
            self._pinned[n:size].zero_()
            dev = torch.empty(size, dtype=torch.uint8, device=self.device)
            dev.copy_(self._pinned[:size], non_blocking=True)
            return dev, n
        buf = torch.zeros(size, dtype=torch.uint8)
        buf[:n].copy_(src)
        return buf, n

    # ------------------------------------------------------------------ matching
    def _start(self, timings) -> float:
        if self.profile:
            TR.start(timings, self.device)
        return 0.0

    def _tick(self, timings, name, t0):
        """Stage boundary: a HIP event on the compute stream (no sync; read in tracing.resolve)."""
        if self.profile:
            TR.mark(timings, name, self.device)
        return t0

    def match_candidates(self, text, nbytes, ls, ll, host_text=None, timings=None,
                         inj: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, int]:
        """(regex << 32 | line) candidates: ``[:pre_from]`` prefilter candidates still to DFA-verify
        (verified inside the post-match pipeline), ``[pre_from:]`` hits of engines that verify
        themselves (literal-free DFA scan, MFMA NFA, the host backtracker's side path). Duplicates
        allowed. ``host_text``: the same bytes on the host (uint8 array), if the caller has them;
        ``inj``: the backtracker side path's keys when the caller ran it (``host_hits``)."""
        timings = {} if timings is None else timings
        if inj is None:
            inj = self.host_hits(text, nbytes, host_text)
        t = self._start(timings)
        cand = K.prefilter(text, nbytes, self.tabs["pf"], ls, self.cand_cap, self.pf_grid)
        t = self._tick(timings, "prefilter", t)
        extra = []
        for sp in self.tabs["scan_passes"]:        # literal-free regexes: multi-regex DFAs in LDS
            extra.append(K.scan_multi(text, nbytes, ls, ll, sp, max(1024, ls.numel() >> 6), self.scan_grid(sp)))
        if self.tabs["scan_regs"].numel():        # one whose DFA alone exceeds a scan group
            extra.append(K.scan(text, ls, ll, self.tabs["scan_regs"], self.tabs["dfa"], max(1024, ls.numel())))
        for ncls, glist in self.tabs["nfa_scan_lists"].items():       # engine.nfa-engine=mfma
            if glist.numel():
                extra.append(K.nfa_scan(self.tabs["nfa_tables"], glist, ncls, text, ls, ll, max(1024, ls.numel())))
        if inj is not None and inj.numel():
            extra.append(inj)
        if extra:
            t = self._tick(timings, "scan", t)
            cand, pre = torch.cat([cand] + extra), cand.numel()
        else:
            pre = cand.numel()
        if self.lib.host_dev:              # relaxation keys: the host side path decided these regexes
            hd = torch.from_numpy(self.lib.host_dev_mask).to(cand.device)
            drop = (cand >= 0) & hd[(cand >> 32).clamp(min=0, max=hd.numel() - 1)]
            if inj is not None and inj.numel():
                drop[cand.numel() - inj.numel():] = False          # (the host side path's own keys)
            cand = torch.where(drop, torch.full_like(cand, -1), cand)
        return cand, pre

    def host_hits(self, text, nbytes: int, host_text=None, ls_h=None, ll_h=None,
                  trim: bool = True, plan=None) -> Optional[torch.Tensor]:
        """The host backtracker's side path (non-regular regexes -- backreferences,
        lookaround, atomic groups, possessive quantifiers -- on C++ BtRegex): run BEFORE the device
        pipeline on the host copy of the bytes, so its verified (regex << 32 | line) keys join the
        device matchers' hits (``match_and_hits(inject=...)``, the native runner's ``inj``) and no
        host round trip, veto of the native runner or of the deferred DP step sits in a batch.
        Lines holding one of a regex's required literals are checked, every line without one.
        ``ls_h`` / ``ll_h``: the batch's host line index (serving), else a Java split of the one
        document / shard (the device line index's rule; ``trim=False``: a stream chunk's rule, no
        trailing-empty-line removal). None without backtracker regexes. ``plan``: the regexes to run
        (default: every backtracker regex; ``lib.host_plan_undev`` when the device feeds the others)."""
        plan = self.lib.host_plan if plan is None else plan
        if not plan:
            return None
        hb = host_text
        if hb is None:
            hb = text[:nbytes].cpu().numpy()
        return torch.from_numpy(self._host_keys(hb, nbytes, ls_h, ll_h, trim, plan)).to(text.device)

    def _host_keys(self, hb, nbytes: int, ls_h=None, ll_h=None, trim: bool = True, plan=None) -> np.ndarray:
        lib = self.lib
        plan = lib.host_plan if plan is None else plan
        hb = np.ascontiguousarray(np.asarray(hb, dtype=np.uint8)[:nbytes])
        if hb.size == 0:
            hb = np.zeros(1, np.uint8)
        if ls_h is not None:
            ls_h = np.ascontiguousarray(ls_h, np.int64)
            ll_h = np.ascontiguousarray(ll_h, np.int32)
            lsp, llp, nl = ls_h.ctypes.data, ll_h.ctypes.data, ls_h.size
        else:
            lsp = llp = nl = 0
        loc, glob, lits = zip(*plan)
        keys = lib.host_bt.prepass(hb.ctypes.data, int(nbytes), lsp, llp, nl, trim, list(loc), list(glob),
                                   [list(x) for x in lits])
        if lib.host_bt.exhausted:
            log.warning("host backtracker: %d line matches exceeded the step budget (treated as no match)",
                        lib.host_bt.exhausted)
        return keys

    def scan_grid(self, sp: tuple) -> int:
        """Persistent grid of k_scan_multi: as many blocks per CU as the pass's LDS blob allows."""
        if self.device.type != "cuda":
            return 0
        # sp[1] = LDS words of the blob; + the 32 KiB lane-replicated bytemap of the 1024-thread blocks
        # (scan_multi.hip SCAN_BM_REP_BYTES): a blob up to 48 KiB gives 2 blocks (8 waves / SIMD with
        # the deferred rare path's <= 64 VGPRs)
        per_cu = max(1, min(2, (160 << 10) // max(sp[1] * 4 + (32 << 10), 1)))
        return self.n_cus * per_cu

    def _ev_tables(self, segs: "Segments") -> tuple:
        return K.ev_tables(self.tabs, segs, len(self.lib.freq_ids), len(self.lib.patterns))

    def match_hits(self, text, nbytes, ls, ll, host_text=None, timings=None) -> torch.Tensor:
        """Sorted unique verified (regex << 32 | line) hit keys of every library regex."""
        cand, pre = self.match_candidates(text, nbytes, ls, ll, host_text, timings)
        segs = Segments.single(ls.numel(), text.device)
        return K.post_hits(cand, pre, ls.numel(), self.lib.n_regexes, text, ls, ll, self.tabs["dfa"],
                           self._ev_tables(segs), self.ws)[0]

    # ------------------------------------------------------------------ core run
    def prefilter_early(self, text, nbytes: int, nlp=None):
        """Queue the literal prefilter before the line index reaches the host (bulk path; pass the
        result to ``prepare(early=...)``). None when the matcher arena path does not apply.
        ``nlp``: the line index's pass-1 outputs -- the prefilter then also writes them (see
        ``fuses_line_index``)."""
        if not text.is_cuda or self.profile:
            return None
        return K.EarlyPrefilter(text, nbytes, self.tabs, self.arena, self.pf_grid, nlp, stream=self._pf_stream)

    def split_with_prefilter(self, text, nbytes: int):
        """Line index + the early literal prefilter -> (ls, ll, early): the prefilter is queued
        behind the line index, before the host's line-count read (on its own stream when the engine
        has one, so the line index's tail and the scans run beside it)."""
        # (starting the prefilter FIRST, beside the whole line index, measured slower: config 2
        # resident 0.506 -> 0.536 ms, bench device step 2.78 -> 2.86 ms -- the line index, which
        # the host waits on, then shares the chip with the prefilter)
        box = []
        ls, ll = K.split_lines(text, nbytes, before_read=(lambda: box.append(self.prefilter_early(text, nbytes)))
                               if text.is_cuda else None, early_first=self._pf_stream is not None)
        return ls, ll, (box[0] if box else None)

    def fuses_line_index(self, text) -> bool:
        """The bulk step folds the line index's first pass into the literal prefilter (one read of the
        text fewer): device text, the arena path, a library with literals. Opt-in
        (``engine.fused-line-index``) until its GPU A/B is in."""
        pf = self.lib.pf
        return (text.is_cuda and not self.profile and bool(self.config.get("engine.fused-line-index", False))
                and bool((pf["gmask"] & 28) or pf["teddy_lits"]))

    def can_defer(self, text) -> bool:
        """``prepare(defer=True)`` applies: device text, every matcher on the arena path, and the
        bucket-sorted post path (csrc/kernels/post_bulk.hip: device-count events)."""
        import os
        return text.is_cuda and not self.profile and self.context_engine != "mfma"

    def prepare(self, text, nbytes, ls, ll, segs: Segments, host_text=None,
                timings: Optional[dict] = None, early=None, defer: bool = False,
                host_index: Optional[tuple] = None, split_trim: bool = True) -> "Prepared":
        """Local phase: matching, hit CSR, events, in-batch frequency ranks, context features.

        Needs no global information, so the data-parallel path runs it before its collectives.
        After matching it is the native post-match pipeline (csrc/kernels/lp_post.hip): one host
        read of (hit, event) counts in the middle, everything else stream-ordered on the device.
        ``defer`` (``can_defer``): no read at all -- hits and events run in device-count mode on
        capacity-sized buffers (``Prepared.cnt`` / ``caps``); the caller reads the counts once its
        whole step is queued and re-runs the step if a buffer overflowed.
        ``host_text`` / ``host_index`` (line starts, lengths): host copies of the batch for the
        backtracker side path (``host_hits``; a multi-document batch needs its index);
        ``split_trim=False``: the lines came from ``split_chunk_lines`` (stream chunks).
        """
        timings = {} if timings is None else timings
        L = ls.numel()
        t = 0.0
        evt = self._ev_tables(segs)
        hs = None
        plan = None
        if self.lib.host_dev and text.is_cuda and host_text is not None:
            # the device feeds the backtracker regexes with relaxed automata: their candidate lines
            # go to the host and the verified keys come back inside the queued step (side_path.hip);
            # the host side path scans the bytes only for regexes without a device relaxation
            if self._host_side is None:
                from .ops.side_path import HostSide
                self._host_side = HostSide(self.lib, text.device,
                                           wait_s=float(self.config.get("engine.side-path-wait-s", 2.0)))
            self._host_side.check()
            if not self._host_side.take_fallback():   # (after a GPU wait timed out: the host-verified path)
                hs = (self._host_side, np.asarray(host_text, dtype=np.uint8))
                plan = self.lib.host_plan_undev
        inj = self.host_hits(text, nbytes, host_text, *(host_index or (None, None)), trim=split_trim, plan=plan)
        if defer:
            hits, hit_line, hit_off, ev_cnt, ev_end, nh_cap, cnt, caps = K.match_and_hits(
                text, nbytes, ls, ll, self.tabs, self.lib.n_regexes, evt, self.arena, self.ws, self.pf_grid,
                self.scan_grid, side=self._side, early=early, defer=True, inject=inj, host_side=hs)
            nkeys = len(self.lib.freq_ids)
            ne_cap = caps["ev"]
            out_buf = K.results_buffer(ne_cap, nkeys, text.device)
            ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_counts, feat, _ = K.post_events(
                hits, nh_cap, ev_cnt, ev_end, ne_cap, L, evt, text, ls, ll, self.tabs["dfa"], nkeys, self.ws,
                ctx_ext=self.lib.ctx_dfa_extent, out=out_buf, dcounts=cnt[3:5], ne_fit=cnt[5:6])
            return Prepared(ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_counts[:max(nkeys, 1)], hits, hit_off,
                            hit_line, feat, L, timings, out_buf=out_buf, cnt=cnt, caps=caps)
        if text.is_cuda:
            # every matcher appends to fixed-capacity device buffers; ONE host read after the CSR
            self._start(timings)
            try:
                hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne = K.match_and_hits(
                    text, nbytes, ls, ll, self.tabs, self.lib.n_regexes, evt, self.arena, self.ws, self.pf_grid,
                    self.scan_grid, tick=(lambda name: self._tick(timings, name, 0.0)) if self.profile else None,
                    side=self._side, early=early, inject=inj, host_side=hs)
            except K.SidePathTimeout:       # settle() armed the host-verified fallback for this re-run
                return self.prepare(text, nbytes, ls, ll, segs, host_text, timings, None, defer, host_index,
                                    split_trim)
            if hs is not None:
                hs[0].check()
        else:
            cand, pre = self.match_candidates(text, nbytes, ls, ll, host_text, timings,
                                              inj=inj if inj is not None else torch.zeros(0, dtype=torch.int64, device=text.device))
            hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne = K.post_hits(
                cand, pre, L, self.lib.n_regexes, text, ls, ll, self.tabs["dfa"], evt, self.ws)
        t = self._tick(timings, "verify_csr", t)
        nkeys = len(self.lib.freq_ids)
        dfa_feats = self.context_engine != "mfma"
        out_buf = K.results_buffer(ne, nkeys, text.device) if text.is_cuda else None
        ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_counts, feat, cov = K.post_events(
            hits, nh, ev_cnt, ev_end, ne, L, evt, text, ls, ll, self.tabs["dfa"], nkeys, self.ws, features=dfa_feats,
            ctx_ext=self.lib.ctx_dfa_extent, out=out_buf)
        if not dfa_feats:           # A/B engine: context features on the MFMA NFA kernel
            lines = torch.nonzero(cov[:L] > 0).flatten().to(torch.int32)
            feat = K.nfa_features(self.tabs["nfa_tables"], lines, L, text, ls, ll, self.tabs["nfa_ctx_list"],
                                  self.lib.nfa_ctx_ncls)
        self._tick(timings, "events_context_freq", t)
        return Prepared(ev_line, ev_pat, ev_seg, ev_rank, ev_fkey, freq_counts[:max(nkeys, 1)], hits, hit_off,
                        hit_line, feat, L, timings, out_buf=out_buf)

    def seq_chain_table(self, prep: "Prepared", own_lo: int, own_hi: int) -> torch.Tensor:
        """Per sequence-event slot: event index still unmatched after this shard (-1 = done)."""
        tabs = self.tabs
        n = self.lib.n_seq_events
        if n == 0:
            return torch.full((1,), -1, dtype=torch.int32, device=prep.hit_off.device)
        out = torch.empty(n, dtype=torch.int32, device=prep.hit_off.device)     # k_seq_chain writes every slot
        dev = prep.hit_off.is_cuda
        s = torch.cuda.current_stream(prep.hit_off.device).cuda_stream if dev else 0
        N.seq_chain(tabs["slot_seq"].data_ptr(), tabs["seq_ev_off"].data_ptr(), tabs["seq_ev_reg"].data_ptr(),
                    prep.hit_off.data_ptr(), prep.hit_line.data_ptr(), int(own_lo), int(own_hi), n,
                    out.data_ptr(), s, dev)
        return out

    def finish(self, prep: "Prepared", segs: Segments, freq_carry: torch.Tensor,
               seq_carry: Optional[torch.Tensor] = None, with_factors: bool = False) -> RunResult:
        """Global phase: fused fp64 score kernel (needs N, global offsets and carries)."""
        timings = dict(prep.timings)
        if TR._MARKS in timings:
            timings[TR._MARKS] = list(timings[TR._MARKS])
        t = self._start(timings)
        tabs = self.tabs
        dev = prep.hit_off.device
        if seq_carry is None:
            seq_carry = torch.zeros(max(self.lib.n_seq_events, 1), dtype=torch.uint8, device=dev)
        st = (tabs["conf"].data_ptr(), tabs["sev"].data_ptr(), tabs["ctx_before"].data_ptr(),
              tabs["ctx_after"].data_ptr(), tabs["sec_off"].data_ptr(), tabs["sec_reg"].data_ptr(),
              tabs["sec_w"].data_ptr(), tabs["sec_weight"].data_ptr(), tabs["seq_off"].data_ptr(),
              tabs["seq_bonus"].data_ptr(), tabs["seq_ev_off"].data_ptr(), tabs["seq_ev_reg"].data_ptr(),
              seq_carry.data_ptr(), prep.hit_off.data_ptr(), prep.hit_line.data_ptr(), prep.feat.data_ptr(),
              segs.lo.data_ptr(), segs.hi.data_ptr(), segs.own_lo.data_ptr(), segs.g0.data_ptr(), segs.n.data_ptr())
        score_out = None
        if prep.out_buf is not None:
            score_out = K.results_views(prep.out_buf, prep.ev_line.numel(), len(self.lib.freq_ids))[0]
        score, factors = K.score_fused(prep.ev_line, prep.ev_pat, prep.ev_seg, prep.ev_rank, prep.ev_fkey,
                                       freq_carry, st, self.sp_tuple, with_factors, out=score_out, dn=prep.ne_dev)
        self._tick(timings, "score", t)
        return RunResult(prep.ev_line, prep.ev_pat, prep.ev_seg, score, factors,
                         prep.freq_counts[:len(self.lib.freq_ids)], prep.hits, prep.hit_off, prep.n_lines, timings,
                         out_buf=prep.out_buf)

    def run(self, text, nbytes, ls, ll, segs: Segments, freq_carry: torch.Tensor,
            seq_carry: Optional[torch.Tensor] = None, host_text=None, with_factors=False,
            timings: Optional[dict] = None) -> RunResult:
        prep = self.prepare(text, nbytes, ls, ll, segs, host_text, timings)
        return self.finish(prep, segs, freq_carry, seq_carry, with_factors)

    def run_document(self, text, nbytes: int, host_text=None, with_factors: bool = False,
                     record: bool = True) -> RunResult:
        """One device-resident document end to end (config 2): line index, matching, events,
        score and the frequency record, with the fewest host round trips -- the literal prefilter
        is queued behind the line index before its one 24-byte read, matching and events run in
        device-count mode (``prepare(defer=True)``), and the counts come back in ONE read at the
        end (a buffer overflow re-runs with the learned capacities, as the bulk step does). The
        frequency window is read before and recorded after the document (AnalysisService.java:
        50-122 for one request)."""
        if not self.can_defer(text):
            ls, ll = K.split_lines(text, nbytes)
            segs = Segments.single(ls.numel(), text.device)
            res = self.run(text, nbytes, ls, ll, segs, self.freq_carry(), host_text=host_text, with_factors=with_factors)
            if record:
                self.commit_frequency(res.freq_counts)
            return res
        ls, ll, early = self.split_with_prefilter(text, nbytes)
        L = ls.numel()
        # (through the engine's pinned upload buffer: a pageable copy would block the host until the
        # queued prefilter is done, with the matchers not yet launched)
        if self._doc_segs is None or self._doc_segs[0] != L:   # (read-only: reused while L repeats)
            self._doc_segs = (L, Segments.scalar(0, L, 0, L, 0, L, text.device, upload=self.upload))
        segs = self._doc_segs[1]
        for attempt in range(4):
            prep = self.prepare(text, nbytes, ls, ll, segs, host_text=host_text, early=early if attempt == 0 else None,
                                defer=True)
            res = self.finish(prep, segs, self.freq_carry(), None, with_factors)
            queued = record and self.freq_on_device and len(self.lib.freq_ids) > 0
            if queued:                           # the record, gated on the device by the capacities,
                c = prep.caps                    # before the read (not behind a host round trip)
                self.freq.record_tensor(res.freq_counts, gate=(prep.cnt, (c["gram"], c["cand"], c["ver"], c["ev"])))
            h = prep.cnt.cpu().tolist()          # the one count read: gram, cand, ver, hits, events
            counts = h[:5]
            if not K.MatchArena.overflow(counts, prep.caps):
                self.arena.learn_deferred(L, counts)
                ne, nh = h[4], h[3]
                res.ev_line, res.ev_pat, res.ev_seg, res.score = (res.ev_line[:ne], res.ev_pat[:ne], res.ev_seg[:ne],
                                                                  res.score[:ne])
                if res.factors is not None:
                    res.factors = res.factors[:ne]
                res.hit_keys = res.hit_keys[:nh]
                if record and not queued:
                    self.commit_frequency(res.freq_counts)
                return res
            self.arena.learn(L, {"gram": h[0], "cand": h[1], "ver": h[2], "ev": h[4]}, overflow=True)
        raise RuntimeError("run_document: buffers still overflowing after re-runs")

    # ------------------------------------------------------------------ request API
    @property
    def freq_on_device(self) -> bool:
        return getattr(self.freq, "device_resident", False)

    def freq_carry(self) -> torch.Tensor:
        if self.freq_on_device:
            c = self.freq.carry_tensor()
            return c if c.device == self.device else c.to(self.device)
        c = self.freq.carry(self.lib.freq_ids)
        if c.size == 0:
            c = np.zeros(1, np.int64)
        return torch.from_numpy(c).to(self.device)

    def commit_frequency(self, counts, veto: Optional[torch.Tensor] = None) -> None:
        """Record this batch's per-id match counts (tensor or host array) in the sliding window.
        ``veto`` (device int64[1], device window only): skip the record when non-zero."""
        if self.freq_on_device:
            if len(counts) and self.lib.freq_ids:
                self.freq.record_tensor(counts if torch.is_tensor(counts) else torch.from_numpy(np.asarray(counts)),
                                        veto=veto)
            return
        if veto is not None and int(veto.item()):
            return
        if len(counts):
            self.freq.record_counts(self.lib.freq_ids, counts.cpu().numpy() if torch.is_tensor(counts) else counts)

    @staticmethod
    def _results_to_host(res: "RunResult"):
        """events (line, pattern, segment: int32; score: f64) + frequency counts (int64) in ONE
        device->host copy (one sync instead of five)."""
        n = res.ev_line.numel()
        if res.out_buf is not None:        # already one buffer (K.results_buffer): no cat
            h = res.out_buf.cpu().numpy()
            k = res.out_buf.numel() - 20 * n
            a, b = 8 * n, 8 * n + k
            return (h[b:b + 4 * n].view(np.int32), h[b + 4 * n:b + 8 * n].view(np.int32),
                    h[b + 8 * n:b + 12 * n].view(np.int32), h[:a].view(np.float64),
                    h[a:a + 8 * len(res.freq_counts)].view(np.int64))
        parts = [res.ev_line.to(torch.int32), res.ev_pat.to(torch.int32), res.ev_seg.to(torch.int32),
                 res.score.contiguous().view(torch.int32), res.freq_counts.to(torch.int64).contiguous().view(torch.int32)]
        h = torch.cat(parts).cpu().numpy()
        return (h[:n], h[n:2 * n], h[2 * n:3 * n], h[3 * n:5 * n].view(np.float64),
                h[5 * n:].view(np.int64))

    @staticmethod
    def score_param_tuple(p) -> tuple:
        """ScoringParams -> the kernels' ScoreParams tuple (csrc/bind.cpp sp_from)."""
        return (p.decay_constant, p.early_bonus_threshold, p.max_early_bonus, p.penalty_threshold,
                p.max_context_factor, p.freq_threshold, p.freq_max_penalty, float(p.freq_window_hours))

    def summary_from_severity(self, sev_hist: np.ndarray, first_pat: Optional[int]) -> dict:
        return summary_from_severity(self.lib, sev_hist, first_pat)

    def summary(self, ev_pat_host: np.ndarray) -> dict:
        if ev_pat_host.size == 0:
            return {"significantEvents": 0, "highestSeverity": "NONE", "severityDistribution": {}}
        dist: Dict[str, int] = {}
        if ev_pat_host.size < 256:       # small requests: no P-sized histogram
            sev = self.lib.severity
            for p in ev_pat_host.tolist():
                s = sev[p]
                dist[s] = dist.get(s, 0) + 1
            counts = None
        else:
            counts = np.bincount(ev_pat_host, minlength=len(self.lib.patterns))
        for p in (np.nonzero(counts)[0] if counts is not None else ()):
            s = self.lib.severity[p]
            dist[s] = dist.get(s, 0) + int(counts[p])
        best_idx, best = -1, None
        for s in dist:
            if s in SEVERITY_ORDER and SEVERITY_ORDER.index(s) > best_idx:
                best_idx, best = SEVERITY_ORDER.index(s), s
        if best is None:
            best = self.lib.severity[int(ev_pat_host[0])]
        return {"significantEvents": int(ev_pat_host.size), "highestSeverity": best, "severityDistribution": dist}

    def analyze_bytes(self, data: bytes, with_factors: bool = False, record: bool = True):
        """One document end to end. Returns (RunResult, host line index arrays)."""
        text, n = self.stage_text(data)
        ls, ll = K.split_lines(text, n)
        segs = Segments.single(ls.numel(), self.device)
        prep = self.prepare(text, n, ls, ll, segs, np.frombuffer(data, np.uint8) if n else None)
        carry = self.freq_carry()
        res = self.finish(prep, segs, carry if record else self._carry_before(BatchJob((), 0.0, recorded=True), prep,
                                                                               carry), with_factors=with_factors)
        if record:
            self.commit_frequency(res.freq_counts)
        return res, ls, ll

    # documents larger than this are line-indexed on the GPU (k_nl_count/k_nl_write); smaller
    # batches are split on the host while they are being packed (memchr, no extra pass)
    GPU_SPLIT_BYTES = 32 << 20

    def analyze_batch_json(self, logs_list: Sequence[str], turn=None, seq: int = 0,
                           record: bool = True) -> List[bytes]:
        """Continuous-batching entry: many requests -> ONE device batch -> one JSON per request.

        Requests become segments of a single line batch (windows never cross a segment, each
        keeps its own N); frequency updates follow the batch (= arrival) order, which is the
        deterministic version of the reference's concurrent-request interleaving. With ``turn``
        (several engines serving concurrently) the frequency carry of batch ``seq`` is read and
        its counts recorded inside the turn; the caller releases the turn on failure.

        = ``pack_batch`` -> ``device_batch`` -> ``emit_batch``; the serving pipeline
        (serve/pipeline.py) runs the three stages of consecutive batches on different threads.
        """
        job = self.pack_batch(logs_list)
        job.recorded = not record          # record=False: a fallback re-run of an already recorded batch
        try:
            self.device_batch(job, turn, seq)
            return self.emit_batch(job)
        finally:
            self.release_batch(job)

    def pack_batch(self, logs_list: Sequence, early_upload: bool = False) -> "BatchJob":
        """Stage 1 (host): pack the request bodies into a pinned staging buffer + line index.
        ``early_upload``: nothing else uses the device half (a lone batch run inline) -- a request
        staged in place has its text queued for upload before the line index is built."""
        t0 = time.time()
        self._batches += 1
        job = BatchJob(logs=logs_list, t0=t0, tm={} if self.profile else None, number=self._batches)
        if len(logs_list) == 1 and len(logs_list[0]) >= self.GPU_SPLIT_BYTES:
            job.whole = True                    # one huge document: streamed by analyze_json
            return job
        job.stage = self._stage_pool.take()
        try:
            with TR.HostTimer(job.tm, "line_index"):
                staged = self._stage_docs(job, logs_list, early_upload)
                if staged is None:              # lone surrogates: encode in Python
                    staged = self._stage_docs(job, [l if isinstance(l, (bytes, bytearray)) else
                                                    l.encode("utf-8", errors="surrogatepass") for l in logs_list])
        except BaseException:
            self.release_batch(job)
            raise
        job.staged = staged
        return job

    def device_batch(self, job: "BatchJob", turn=None, seq: int = 0) -> None:
        """Stage 2 (device): H2D, match + score kernels, one D2H, frequency commit (in batch order)."""
        if self.fault_every and job.number % self.fault_every == 0:
            raise RuntimeError("injected device fault (engine.fault-inject-every)")
        self._device_batch(job, turn, seq)
        if self.fault_after_record and job.number % self.fault_after_record == 0:
            raise RuntimeError("injected device fault after the frequency record (engine.fault-inject-after-record)")

    def _device_batch(self, job: "BatchJob", turn=None, seq: Optional[int] = 0) -> None:
        """``seq`` None (serving processes): the batch draws its arrival ticket from ``turn`` itself,
        as late as its path allows, and releases it on every exit."""
        if job.whole:
            if turn is not None:
                if seq is None:
                    seq = turn.take()
                turn.wait(seq)
            try:
                doc = job.logs[0]
                job.outs = [self.analyze_json(doc.decode() if isinstance(doc, N.RawLogs) else doc,
                                              record=not job.recorded)]
                job.recorded = True
                if turn is not None:
                    self._window_quiet()
            finally:
                if turn is not None:
                    turn.done(seq)
            return
        hb, ls_h, ll_h, dl, n = job.staged
        tm = job.tm
        verbose = self.log_matches or log.isEnabledFor(logging.DEBUG)
        if (turn is None or isinstance(turn, SharedWindowTurn)) and self._runner_ok(job, verbose, tm):
            # the whole device half in one native call (csrc/runtime/request.cpp); with a shared
            # window its eviction / score / record run in arrival order inside the runner
            self._run_native(job, dl, n, turn, seq)
            return
        if tm is not None:
            self._start(tm)
        text = self._stage_h2d(job.stage.buf, n)
        lo, hi, g0, nn = Segments.doc_arrays(dl)
        pinned_idx = job.n_lines >= 0 and self.device.type == "cuda"
        if pinned_idx:                     # line index straight from the pinned stage (no host copy)
            ls = job.stage.starts(job.n_lines).to(self.device, non_blocking=True)
            ll = job.stage.lens(job.n_lines).to(self.device, non_blocking=True)
            idx = []
        else:
            idx = [ls_h, ll_h]
        if turn is None and self.freq_on_device:
            # the window lives in HBM: carry read and counts recorded on the device, no host trip
            up = self.upload(idx + [lo, hi, g0, nn])
            if not pinned_idx:
                ls, ll = up[0], up[1]
            lo, hi, g0, nn = up[len(idx):]
            segs = Segments(lo, hi, lo, hi, g0, nn)
            if tm is not None:
                self._tick(tm, "h2d", 0.0)
            res = self._run_job(job, text, n, ls, ll, segs, self.freq_carry(), hb[:n], verbose, tm, (ls_h, ll_h))
            if not job.recorded:
                self.commit_frequency(res.freq_counts)
                job.recorded = True
            with TR.HostTimer(tm, "d2h"):
                job.ev = self._results_to_host(res)
        elif turn is None:
            carry = self.freq.carry(self.lib.freq_ids)
            up = self.upload(idx + [lo, hi, g0, nn, carry if carry.size else np.zeros(1, np.int64)])
            if not pinned_idx:
                ls, ll = up[0], up[1]
            lo, hi, g0, nn, carry = up[len(idx):]
            segs = Segments(lo, hi, lo, hi, g0, nn)
            if tm is not None:
                self._tick(tm, "h2d", 0.0)
            res = self._run_job(job, text, n, ls, ll, segs, carry, hb[:n], verbose, tm, (ls_h, ll_h))
            with TR.HostTimer(tm, "d2h"):
                job.ev = self._results_to_host(res)
            if not job.recorded:
                self.commit_frequency(job.ev[4])
                job.recorded = True
        else:
            up = self.upload(idx + [lo, hi, g0, nn])
            if not pinned_idx:
                ls, ll = up[0], up[1]
            lo, hi, g0, nn = up[len(idx):]
            segs = Segments(lo, hi, lo, hi, g0, nn)
            if tm is not None:
                self._tick(tm, "h2d", 0.0)
            prep = self.prepare(text, n, ls, ll, segs, host_text=hb[:n], timings=tm, host_index=(ls_h, ll_h))
            if seq is None:                    # serving processes: the ticket once matching is queued
                if self.device.type == "cuda":
                    torch.cuda.current_stream(self.device).synchronize()
                seq = turn.take()
            turn.wait(seq)                     # earlier batches have recorded their counts
            try:
                res = self.finish(prep, segs, self._carry_before(job, prep, self.freq_carry()), with_factors=verbose)
                with TR.HostTimer(tm, "d2h"):
                    job.ev = self._results_to_host(res)
                if not job.recorded:
                    self.commit_frequency(job.ev[4])
                    job.recorded = True
                self._window_quiet()           # the record has landed before later batches evict
            finally:
                turn.done(seq)
        if verbose:
            self._log_events(res, dl)
        if tm is not None:
            job.timings = res.timings

    @staticmethod
    def _carry_before(job: "BatchJob", prep: "Prepared", carry: torch.Tensor) -> torch.Tensor:
        """The carry this batch must be scored with. A re-run of a batch whose counts already
        entered the window (a failure after the record) takes them back out: the penalty is the
        one before its own record (ScoringService.java:84-88)."""
        if not job.recorded or not carry.numel():
            return carry
        k = min(carry.numel(), prep.freq_counts.numel())
        c = carry.clone()
        c[:k] = (c[:k] - prep.freq_counts[:k].to(c.device, c.dtype)).clamp(min=0)
        return c

    def _run_job(self, job: "BatchJob", text, n, ls, ll, segs, carry, host_text, verbose, tm,
                 host_index=None) -> RunResult:
        prep = self.prepare(text, n, ls, ll, segs, host_text, tm, host_index=host_index)
        return self.finish(prep, segs, self._carry_before(job, prep, carry), with_factors=verbose)

    def _window_quiet(self) -> None:
        """Wait for the frequency window's queued kernels (a shared device window: the next batch
        in arrival order may run on another stream or GPU)."""
        if self.freq_on_device and self.freq.device.type == "cuda":
            torch.cuda.current_stream(self.freq.device).synchronize()

    def _runner_ok(self, job: "BatchJob", verbose: bool, tm) -> bool:
        """The native request runner covers the common device configuration: a GPU engine with a
        device-resident frequency window (its own, or one shared by several engines), DFA context
        features, no host-fallback or MFMA scan regexes, the line index in the pinned stage, no
        tracing / per-match logging, a batch not yet recorded."""
        if self._runner is False or tm is not None or verbose or job.n_lines < 0 or job.recorded:
            return False
        if self._runner is None:
            from .frequency import SharedFrequencyState
            hostwin = isinstance(self.freq, SharedFrequencyState)      # serving processes' host window
            ok = (self.device.type == "cuda" and (self.freq_on_device or hostwin)
                  and self.context_engine != "mfma" and bool(self.config.get("engine.native-runner", True))
                  and not any(g.numel() for g in self.tabs["nfa_scan_lists"].values()))
            if not ok:
                self._runner = False
                return False
            t = self.tabs
            ptr = lambda k: t[k].data_ptr()  # noqa: E731
            st12 = tuple(ptr(k) for k in ("conf", "sev", "ctx_before", "ctx_after", "sec_off", "sec_reg", "sec_w",
                                          "sec_weight", "seq_off", "seq_bonus", "seq_ev_off", "seq_ev_reg"))
            ev5 = tuple(ptr(k) for k in ("prim_off", "prim_pats", "freq_key", "ctx_before", "ctx_after"))
            dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
            self._runner = N.RequestRunner(
                t["pf"], t["dfa"], list(t["scan_passes"]), [self.scan_grid(sp) for sp in t["scan_passes"]],
                ptr("scan_regs"), t["scan_regs"].numel(), st12, self.sp_tuple, ev5, self.lib.n_regexes,
                len(self.lib.patterns), len(self.lib.freq_ids), self.lib.n_seq_events, self.lib.ctx_dfa_extent[0],
                self.lib.ctx_dfa_extent[1], self.pf_grid, dev,
                bool(self.config.get("engine.runner-device-counts", True)), bool(self.lib.host_dev))
        return True

    def _run_native(self, job: "BatchJob", dl, n: int, turn: Optional[SharedWindowTurn] = None,
                    seq: Optional[int] = 0) -> None:
        """Engine.device_batch through N.RequestRunner: same kernels and order as prepare / finish
        (H2D, eviction, matchers, ONE counter read, events + features + ranks, score, record,
        ONE results read); the frequency state's host bookkeeping stays here, under its lock.

        With a shared window (``turn``): the bookkeeping runs in arrival order (``turn.host``) and
        only briefly; the runner queues its matchers, then enters the window section through
        ``turn.dev`` -- engines on other GPUs / streams overlap everything but that section.

        The serving processes' host window (``SharedFrequencyState``): the runner itself draws the
        arrival ticket once the batch's carry-independent stages have finished, and evicts / reads
        the carry / records on the host inside its section (``RequestRunner.run(hw=...)``)."""
        lo, hi, g0, nn = Segments.doc_arrays(dl)
        fr = self.freq
        K = len(self.lib.freq_ids)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        st = job.stage
        args = (st.buf.data_ptr(), n, st.starts(job.n_lines).data_ptr(), st.lens(job.n_lines).data_ptr(), job.n_lines,
                lo, hi, g0, nn)
        inj = np.zeros(0, np.int64)
        if self.lib.host_plan:              # the backtracker's side path, on the pinned host bytes
            inj = self._host_keys(st.buf[:n].numpy(), n, st.starts(job.n_lines).numpy(), st.lens(job.n_lines).numpy())
        win = getattr(fr, "win", None)
        if win is not None:                 # the node's host window (serving processes)
            try:
                ne, out, counts, E = self._runner.run(*args, (), 0.0, fr.clock(), stream, st.buf.numel(), inj=inj,
                                                      hw=win, pre_token=job.pre_token)
            except BaseException:
                job.recorded = bool(self._runner.recorded)
                raise
        elif turn is None:
            with fr._lock:
                if K:
                    fr._ensure_room(K)
                evict_before = fr._now() - fr.window_s      # carry_tensor()
                now = fr._now()                              # record_tensor()
                # host_cap: the stage's room behind the text lets the runner send text, line index,
                # segments and zeroed counters in ONE H2D copy (request.cpp, single-copy layout)
                ne, out, counts, E = self._runner.run(*args, fr._ring(), evict_before, now, stream, st.buf.numel(),
                                                      inj=inj, pre_token=job.pre_token)
                if K:
                    fr._tail_bound += K
        else:
            turn.host.wait(seq)
            try:
                with fr._lock:
                    if K:
                        fr._ensure_room(K, quiesce=lambda: turn.dev.wait(seq))
                    evict_before = fr._now() - fr.window_s
                    now = fr._now()
                    ring = fr._ring()
                    if K:
                        fr._tail_bound += K
            finally:
                turn.host.done(seq)
            try:
                ne, out, counts, E = self._runner.run(*args, ring, evict_before, now, stream, st.buf.numel(),
                                                      turn=turn.dev, seq=seq, inj=inj, pre_token=job.pre_token)
            except BaseException:
                job.recorded = bool(self._runner.recorded)
                raise
        job.recorded = True
        self.arena.last = counts
        need = self._runner.upload_bytes(n, job.n_lines, len(lo))
        if need > st.buf.numel():
            st.want = need * 5 // 4                      # grown on release (emission still reads buf)
        k1 = max(K, 1)
        a, b = 8 * E, 8 * E + 8 * k1          # E: the results' event stride (>= ne)
        job.ev = (out[b:b + 4 * ne].view(np.int32), out[b + 4 * E:b + 4 * E + 4 * ne].view(np.int32),
                  out[b + 8 * E:b + 8 * E + 4 * ne].view(np.int32), out[:8 * ne].view(np.float64),
                  out[a:a + 8 * K].view(np.int64))

    def emit_batch(self, job: "BatchJob") -> List[bytes]:
        """Stage 3 (host): every response of the batch (uuid, metadata, events with context lines,
        summary) in one native call with the GIL released (csrc/io/json_emit.cpp)."""
        if job.outs is not None:
            return job.outs
        hb, ls_h, ll_h, dl, n = job.staged
        ev_line, ev_pat, ev_seg, score, _ = job.ev
        ndocs = len(job.logs)
        extra = b""
        if job.tm is not None:
            import json
            st = {k: round(v, 4) for k, v in TR.resolve(job.timings).items()}
            st.update({k: round(v, 4) for k, v in TR.resolve(job.tm).items()})
            st["batchRequests"] = ndocs
            log.debug("stage timings (ms): %s", st)
            extra = (',"stageTimingsMs":' + json.dumps(st, separators=(",", ":"))).encode()
        now, ts = self._clock()
        bounds = np.searchsorted(ev_seg, np.arange(ndocs + 1)).astype(np.int64)
        tail = f',"analyzedAt":"{ts}","patternsUsed":{self._patterns_used()}'.encode() + extra
        return N.emit_batch_results(self._pattern_table(), hb.ctypes.data, ls_h, ll_h,
                                    np.ascontiguousarray(dl, np.int64), ev_line, ev_pat, score, bounds,
                                    int((now - job.t0) * 1000), tail, self._STAGE_THREADS)

    def release_batch(self, job: "BatchJob") -> None:
        """Return the job's staging buffer to the pool (after its H2D and emission are done)."""
        if job.stage is not None:
            if job.stage.own_buf is not None:   # staged in place in a request's pinned buffer
                job.stage.buf, job.stage.own_buf = job.stage.own_buf, None
                job.stage.want = 0
            if job.stage.want > job.stage.buf.numel():
                try:
                    job.stage.grow_buf(job.stage.want)
                except BaseException:           # keep the slot usable; the next pack regrows
                    job.stage.buf = None
            self._stage_pool.give(job.stage)
            job.stage = None

    _STAGE_THREADS = host_thread_budget()
    inplace_stages = 0          # batches staged in place in a request's pinned decode buffer
    _pinned_views: dict = {}    # (address, capacity) of a pinned decode buffer -> its uint8 tensor view

    def _stage_docs(self, job: "BatchJob", docs, early_upload: bool = False):
        """Pack request bodies into the job's (pinned) staging buffer and build the per-document
        line index, in native code with the GIL released (csrc/io/docs.cpp): one host copy per
        byte; the index goes straight into the stage's pinned index buffer when it fits.
        Returns (host view, line_start, line_len, doc_line_off, nbytes) or None."""
        st = job.stage
        raw = [isinstance(d, N.RawLogs) for d in docs]
        if any(raw) and not all(raw):   # escaped request logs are unescaped in place only as a batch
            docs = [d.decode() if r else d for d, r in zip(docs, raw)]
        r = None
        if len(docs) == 1 and raw[0] and self.device.type == "cuda":
            # decoded by the HTTP IO thread into a pinned buffer: that buffer IS this batch's stage
            # (the decoder recorded its newlines, so packing is the line index alone; the runner
            # uploads from it and the emitter reads it). The RawLogs in job.logs keeps it alive.
            addr, pcap = docs[0].pinned_text
            if addr:
                if early_upload and self._runner:
                    # the text is final: its upload runs while the line index is built (RequestRunner
                    # .prefetch_text; run(pre_token=) then sends only what follows the text)
                    job.pre_token = self._runner.prefetch_text(addr, docs[0].decoded_len, pcap,
                                                               torch.cuda.current_stream(self.device).cuda_stream)
                r = N.pack_split_docs(docs, addr, pcap - K.TEXT_PAD - K.NL_TILE, self._STAGE_THREADS,
                                      st.idx.data_ptr(), st.cap)
                if isinstance(r, tuple) and r[1] is None:
                    st.own_buf = st.buf
                    views = self._pinned_views       # (the server recycles a few such buffers)
                    v = views.get((addr, pcap))
                    if v is None:
                        if len(views) > 32:
                            views.clear()
                        v = views[(addr, pcap)] = torch.from_dlpack(N.dlpack(addr, pcap, "uint8", -1))
                    st.buf = v
                    self.inplace_stages += 1
                else:
                    r = None
        if r is None:
            cap = st.buf.numel() - K.TEXT_PAD - K.NL_TILE
            r = N.pack_split_docs(docs, st.buf.data_ptr(), cap, self._STAGE_THREADS, st.idx.data_ptr(), st.cap)
        if r is None:
            return None
        if isinstance(r, int):
            # geometric: a burst's batches grow from a few requests to thousands, and every
            # re-pinning of a 100+ MB stage costs tens of ms on the serving path (profiles/r4_b)
            size = K.padded_len(max(int(r) * 5 // 4, 2 * st.buf.numel(), 1 << 20))
            st.grow_buf(size)
            r = N.pack_split_docs(docs, st.buf.data_ptr(), size - K.TEXT_PAD - K.NL_TILE, self._STAGE_THREADS,
                                  st.idx.data_ptr(), st.cap)
        a, ll_h, dl, doc_off = r
        if ll_h is None:                   # index written into the stage
            job.n_lines = int(a)
            ls_h, ll_h = st.starts(job.n_lines).numpy(), st.lens(job.n_lines).numpy()
        else:
            ls_h = a
            job.n_lines = -1
            st.grow_idx(max(ls_h.size * 5 // 4, 2 * st.cap))  # fits next time
        n = int(doc_off[-1])
        return st.buf.numpy(), ls_h, ll_h, dl, n

    def _stage_h2d(self, buf: torch.Tensor, n: int) -> torch.Tensor:
        size = K.padded_len(n)
        buf[n:size].zero_()
        if self.device.type == "cuda":
            dev = torch.empty(size, dtype=torch.uint8, device=self.device)
            dev.copy_(buf[:size], non_blocking=True)
            return dev
        return buf[:size]

    def _log_events(self, res: RunResult, doc_line_off) -> None:
        """Reference-style match / factor logs (AnalysisService.java:96-99 INFO per match,
        ScoringService.java:90-99 DEBUG factor breakdown); opt-in via server.log-matches or DEBUG."""
        ev_line = res.ev_line.cpu().numpy()
        ev_pat = res.ev_pat.cpu().numpy()
        ev_seg = res.ev_seg.cpu().numpy()
        fac = res.factors.cpu().numpy() if res.factors is not None else None
        lvl = logging.INFO if self.log_matches else logging.DEBUG
        for e in range(ev_line.size):
            pat = self.lib.patterns[int(ev_pat[e])]
            ln = int(ev_line[e] - doc_line_off[ev_seg[e]]) + 1
            log.log(lvl, "Line %d: Found match for pattern '%s'", ln, pat.name)
            if fac is not None and log.isEnabledFor(logging.DEBUG):
                f = fac[e]
                log.debug("Pattern '%s': Base Confidence=%s, Severity Multiplier=%s, Chronological Factor=%s, "
                          "Proximity Factor=%s, Temporal Factor=%s, Context Factor=%s, Frequency Penalty=%s",
                          pat.name, *[float(x) for x in f])

    def _pattern_table(self):
        pt = getattr(self.lib, "_native_pattern_table", None)
        if pt is None:
            pt = N.PatternTable(self.lib.pattern_json, self.lib.ctx_before, self.lib.ctx_after)
            rank = np.array([SEVERITY_ORDER.index(s) if s in SEVERITY_ORDER else -1 for s in self.lib.severity],
                            np.int32)
            pt.set_severity(list(self.lib.severity), rank)
            self.lib._native_pattern_table = pt
        return pt

    def _patterns_used(self) -> str:
        pu = getattr(self, "_patterns_used_json", None)
        if pu is None:
            import json
            pu = self._patterns_used_json = json.dumps(self.lib.library_ids, separators=(",", ":"))
        return pu

    def analyze_json(self, logs, library_ids: Optional[List] = None, record: bool = True) -> bytes:
        """Full AnalysisResult as JSON bytes (camelCase result, snake_case matchedPattern)."""
        data = logs if isinstance(logs, (bytes, bytearray)) else logs.encode("utf-8", errors="surrogatepass")
        if len(data) < self.GPU_SPLIT_BYTES:
            return self.analyze_batch_json([logs], record=record)[0]
        t0 = time.time()
        res, ls, ll = self.analyze_bytes(data, record=record)
        ev_line = res.ev_line.cpu().numpy()
        ev_pat = res.ev_pat.cpu().numpy()
        score = res.score.cpu().numpy()
        ls_h = ls.cpu().numpy()
        ll_h = ll.cpu().numpy()
        buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        events_json = N.emit_events_json(self._pattern_table(), buf.ctypes.data, ls_h, ll_h, 0, int(ls_h.size),
                                         ev_line, ev_pat, score)
        return self._wrap(events_json, ev_pat, int(ls_h.size), t0)

    @staticmethod
    def _clock() -> tuple:
        now = time.time()
        return now, datetime.fromtimestamp(now, timezone.utc).isoformat().replace("+00:00", "Z")

    _EMPTY_SUMMARY = b',"summary":{"significantEvents":0,"highestSeverity":"NONE","severityDistribution":{}}}'

    def _wrap(self, events_json: bytes, ev_pat: np.ndarray, total_lines: int, t0: float,
              extra_meta: bytes = b"", clock: Optional[tuple] = None) -> bytes:
        """AnalysisResult JSON around the natively emitted events array (AnalysisService.java:115-121).
        ``clock`` = (now, ISO timestamp) shared by every request of a batch (they finish together)."""
        import json
        pu = self._patterns_used()
        now, ts = clock if clock is not None else self._clock()
        head = (f'{{"analysisId":"{uuid.uuid4()}","metadata":{{"processingTimeMs":{int((now - t0) * 1000)},'
                f'"totalLines":{total_lines},"analyzedAt":"{ts}","patternsUsed":{pu}').encode() \
            + extra_meta + b'},"events":'
        if ev_pat.size == 0:
            return head + events_json + self._EMPTY_SUMMARY
        summ = json.dumps(self.summary(ev_pat), separators=(",", ":"))
        return head + events_json + (',"summary":' + summ + "}").encode()

    def analyze(self, logs: str) -> dict:
        import json
        return json.loads(self.analyze_json(logs))
