"""Host half of the device-fed backtracker regexes (csrc/kernels/side_path.hip).

A backtracker regex (backreference, lookaround, atomic group, possessive quantifier: the regexes
``java.util.regex`` needs a backtracker for, ``AnalysisService.java:88-95``) carries, on the device,
the automaton of its regular relaxation (``jregex.cpp Relaxer``). In a bulk step its device keys are
candidates: ``k_take_host`` exports them (key, line start, length) to pinned host memory, a helper
thread (native: bind.cpp SideWorker) checks the lines with the C++ backtracker on the step's host bytes and publishes the
verified keys, and ``k_wait_host`` -- queued behind the export, so the rest of the step is queued
with no host round trip -- appends them to the verified-hit buffer. The host only ever looks at
candidate lines: never the whole shard, and never a device-to-host copy of the text.

Failure handling: the helper always publishes (a count of -1 on an error or an export that
overflowed its buffer); ``k_wait_host`` then overflows the verified-hit buffer, so the batch's
frequency record is vetoed and the caller re-runs it -- with a larger export buffer, or raising the
helper's error (``check``).
"""
from __future__ import annotations

import logging

import numpy as np
import torch

from ..native import N

log = logging.getLogger("log_parser_amd.side_path")


class _Coherent:
    """Fine-grained pinned host memory: (host numpy view, device address)."""

    def __init__(self, n: int):
        self.h, self.d = N.host_alloc_coherent(8 * n)
        self.a = torch.from_dlpack(N.dlpack(self.h, n, "int64", -1)).numpy()


class HostSide:
    def __init__(self, lib, device: torch.device, cap: int = 1 << 14):
        self.lib = lib
        self.device = device
        self.seq = 0
        self.cnt = torch.zeros(2, dtype=torch.int64, device=device)   # [export count, done blocks]
        self._alloc(cap)
        # the verifying thread is native (bind.cpp SideWorker): no GIL between export and answer
        self._worker = N.SideWorker(lib.host_bt, [int(x) for x in np.asarray(lib.host_local, np.int32)])
        self._hold = []                            # host bytes of the queued batches (the worker reads them)

    def _alloc(self, cap: int) -> None:
        self.cap = int(cap)
        self.out = _Coherent(3 * self.cap + 2)     # keys | starts | lens | host count | host seq
        self.inb = _Coherent(self.cap + 3)         # keys | host count | host seq | err

    @property
    def need(self) -> int:
        return int(self._worker.need)

    def queue(self, cand, n1d: int, cap1: int, ver, n2d: int, cap2: int, text, ls, ll, dfa, stream: int,
              host_text: np.ndarray) -> None:
        """Queue export -> (host verification) -> append on ``stream``; host_text: the batch's
        bytes on the host (the offsets of ``ls`` index it), read by the worker until it publishes
        (the batch's end-of-step read comes after k_wait_host, hence after that)."""
        need = self.need
        if need > self.cap:                        # (the previous attempt's buffers are idle)
            self._alloc(max(need * 5 // 4, 2 * self.cap))
            self._worker.clear_need()
        self.seq += 1
        c, o, i = self.cap, self.out.d, self.inb.d
        N.take_host(cand.data_ptr(), n1d, cap1, ver.data_ptr(), n2d, cap2, text.data_ptr(), ls.data_ptr(),
                    ll.data_ptr(), dfa, (o, o + 8 * c, o + 16 * c, c, self.cnt.data_ptr(), self.cnt.data_ptr() + 8,
                                         o + 24 * c, o + 24 * c + 8, self.seq), stream)
        ht = np.ascontiguousarray(host_text)
        self._hold = (self._hold + [ht])[-4:]
        self._worker.submit(self.seq, ht.ctypes.data, c, self.out.h, self.inb.h)
        N.wait_host(ver.data_ptr(), cap2, n2d, (i, i + 8 * c, i + 8 * c + 8, c, self.seq, i + 8 * c + 16), stream)

    def check(self) -> None:
        """Raise the helper's error (the step has re-run or failed meanwhile)."""
        e = self._worker.take_error()
        if e:
            log.error("backtracker side path failed: %s", e)
            raise RuntimeError(f"backtracker side path failed: {e}")
