"""Host half of the device-fed backtracker regexes (csrc/kernels/side_path.hip).

A backtracker regex (backreference, lookaround, atomic group, possessive quantifier: the regexes
``java.util.regex`` needs a backtracker for, ``AnalysisService.java:88-95``) carries, on the device,
the automaton of its regular relaxation (``jregex.cpp Relaxer``). In a bulk step its device keys are
candidates: ``k_take_host`` exports them (key, line start, length) to pinned host memory -- the
prefilter's candidates as soon as the literal chain is done, the scan engines' keys after the scan --
a helper thread (native: bind.cpp SideWorker) checks the lines with the C++ backtracker on the
step's host bytes and publishes the verified keys, and ``k_wait_host`` -- queued behind the export, so the rest of the step is queued
with no host round trip -- appends them to the verified-hit buffer. The host only ever looks at
candidate lines: never the whole shard, and never a device-to-host copy of the text.

Failure handling: the helper always publishes (a count of -1 on an error or an export that
overflowed its buffer); ``k_wait_host`` then overflows the verified-hit buffer, so the batch's
frequency record is vetoed and the caller re-runs it -- with a larger export buffer, or raising the
helper's error (``check``). When the GPU stopped waiting (the host's verification of a large step
took longer than ``wait_s``), the re-run does not go through the same wait again: ``settle`` arms a
one-step FALLBACK, and the engine re-runs that step on the host-verified path (``Engine.host_hits``
over every backtracker regex before the device work, the relaxation keys only dropped), which is
slower but has no GPU-side deadline; the GPU's wait for later steps is doubled (up to
``max_wait_s``).
"""
from __future__ import annotations

import logging

import numpy as np
import torch

from ..native import N

log = logging.getLogger("log_parser_amd.side_path")


class _Coherent:
    """Fine-grained pinned host memory: (host numpy view, device address); freed by ``free``."""

    def __init__(self, n: int):
        self.h, self.d = N.host_alloc_coherent(8 * n)
        self.a = torch.from_dlpack(N.dlpack(self.h, n, "int64", -1)).numpy()

    def free(self) -> None:
        if self.h:
            self.a = None
            N.host_free_coherent(self.h)
            self.h = self.d = 0


class HostSide:
    """The device side of one engine's exports: pinned regions A (prefilter candidates) and B (the
    scan engines' relaxation keys), the verified-key buffer the GPU appends from, and the native
    verifying thread."""

    def __init__(self, lib, device: torch.device, cap: int = 1 << 14, wait_s: float = 2.0,
                 max_wait_s: float = 30.0):
        self.lib = lib
        self.device = device
        self.seq = 0
        self.cnt = torch.zeros(4, dtype=torch.int64, device=device)   # [count, done blocks] x (A, B)
        self.wait_s = float(wait_s)                # k_wait_host's wall-clock limit (doubled per timeout)
        self.max_wait_s = float(max_wait_s)
        self._fallback = False                     # the next step runs on the host-verified path
        self._retired = []                         # (buffers, seq): superseded, freed once the worker is past seq
        self.out_a = self.out_b = self.inb = None
        self._alloc(cap)
        # the verifying thread is native (bind.cpp SideWorker): no GIL between export and answer
        self._worker = N.SideWorker(lib.host_bt, [int(x) for x in np.asarray(lib.host_local, np.int32)])
        self._hold = []                            # host bytes of the queued batches (the worker reads them)
        self.waits_failed = 0                      # jobs the GPU stopped waiting for (settle)
        self.fallbacks = 0                         # steps re-run on the host-verified path

    def _alloc(self, cap: int) -> None:
        if self.out_a is not None:                 # a queued job may still read / write the old regions
            self._retired.append(((self.out_a, self.out_b, self.inb), self.seq))
        self.cap = int(cap)
        self.out_a = _Coherent(3 * self.cap + 2)   # keys | starts | lens | host count | host seq
        self.out_b = _Coherent(3 * self.cap + 2)
        self.inb = _Coherent(self.cap + 3)         # keys | host count | host seq | err
        self._reap()

    def _reap(self) -> None:
        """Free superseded regions the worker has answered every job of."""
        done = int(self._worker.done) if hasattr(self, "_worker") else -1
        keep = []
        for bufs, seq in self._retired:
            if done >= seq:
                for b in bufs:
                    b.free()
            else:
                keep.append((bufs, seq))
        self._retired = keep

    def close(self) -> None:
        """Free every region once the worker has answered its jobs (engine shutdown)."""
        self.settle(strict=False)
        self._retired.append(((self.out_a, self.out_b, self.inb), self.seq))
        self._reap()

    def take_fallback(self) -> bool:
        """True once after a GPU wait timed out: the caller runs this step on the host-verified path."""
        f, self._fallback = self._fallback, False
        if f:
            self.fallbacks += 1
        return f

    @property
    def need(self) -> int:
        return int(self._worker.need)

    def _out(self, o, k: int) -> tuple:
        c, d = self.cap, o.d
        cnt = self.cnt.data_ptr() + 16 * k
        return (d, d + 8 * c, d + 16 * c, c, cnt, cnt + 8, d + 24 * c, d + 24 * c + 8, self.seq)

    def begin(self, host_text: np.ndarray) -> None:
        """A new job (one attempt of a step): buffers sized for the worker's last request, a new
        sequence number, the worker told where the step's host bytes are (``ls`` offsets index them;
        it reads them until it publishes, and the step's end-of-step read comes after that)."""
        need = self.need
        if need > self.cap:                        # (the previous attempt's buffers are idle)
            self._alloc(max(need * 5 // 4, 2 * self.cap))
            self._worker.clear_need()
        elif self._retired:
            self._reap()
        self.seq += 1
        ht = np.ascontiguousarray(host_text)
        self._hold = (self._hold + [ht])[-4:]
        self._worker.submit(self.seq, ht.ctypes.data, self.cap, self.out_a.h, self.out_b.h, self.inb.h)

    def export_scan(self, ver, n2d: int, cap2: int, text, ls, ll, dfa, stream: int) -> None:
        """Region B, queued on the scans' stream as soon as they end: the scan engines' keys of
        relaxed regexes go to the host, which verifies them while the literal chain still runs."""
        N.take_host(0, 0, 0, ver.data_ptr(), n2d, cap2, text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa,
                    self._out(self.out_b, 1), stream)

    def export_candidates(self, cand, n1d: int, cap1: int, text, ls, ll, dfa, stream: int) -> None:
        """Region A, queued right after the literal chain: the prefilter candidates of relaxed
        regexes leave the candidate buffer for the host (the worker verifies the regions in the
        order their exports arrive)."""
        N.take_host(cand.data_ptr(), n1d, cap1, 0, 0, 0, text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa,
                    self._out(self.out_a, 0), stream)

    def wait(self, ver, n2d: int, cap2: int, stream: int) -> None:
        """k_wait_host, queued after both exports (and after the scans joined): the verified keys of
        both regions are appended to the verified-hit buffer."""
        c, i = self.cap, self.inb.d
        N.wait_host(ver.data_ptr(), cap2, n2d, (i, i + 8 * c, i + 8 * c + 8, c, self.seq, i + 8 * c + 16), stream,
                    self.wait_s)

    def settle(self, timeout_s: float = 600.0, strict: bool = True) -> int:
        """Before an overflowing step re-runs: wait until the worker has answered every queued job
        (a re-run's export reuses the regions, and a job still reading them would see the next
        attempt's sequence numbers), then return and clear the GPU's wait status of the last job
        (0 answered, 1 no answer within the GPU's wait, 2 the host answered -1). A GPU wait that
        timed out arms the host-verified fallback for the re-run and doubles the GPU's wait.
        ``strict``: raise when the worker has not caught up within ``timeout_s`` (the regions would
        be reused under a running job)."""
        import time
        t0 = time.monotonic()
        while int(self._worker.done) < self.seq and time.monotonic() - t0 < timeout_s:
            time.sleep(0.0005)
        if int(self._worker.done) < self.seq and strict:
            raise RuntimeError(f"backtracker side path: worker still on job {int(self._worker.done) + 1} of "
                               f"{self.seq} after {timeout_s:.0f} s")
        err = int(self.inb.a[self.cap + 2])
        if err:
            self.waits_failed += 1
            log.warning("backtracker side path: job %d %s (worker done %d); the step re-runs%s", self.seq,
                        "not answered within the GPU's wait" if err == 1 else "answered -1 (export overflow)",
                        int(self._worker.done), " on the host-verified path" if err == 1 else "")
            self.inb.a[self.cap + 2] = 0
            if err == 1:
                self._fallback = True
                self.wait_s = min(self.max_wait_s, 2.0 * self.wait_s)
        self._reap()
        return err

    def check(self) -> None:
        """Raise the helper's error (the step has re-run or failed meanwhile)."""
        e = self._worker.take_error()
        if e:
            log.error("backtracker side path failed: %s", e)
            raise RuntimeError(f"backtracker side path failed: {e}")
