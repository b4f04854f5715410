"""Persistent sliding-window frequency state (reference ``FrequencyTrackingService.java:20-162``).

The reference keeps a process-global ``ConcurrentHashMap<patternId, PatternFrequency>`` that
survives across requests (``FrequencyTrackingService.java:25``) and computes a pattern's
penalty from its hourly rate *before* recording the current match (``ScoringService.java:84-88``).

Here the state is vectorised over id slots: a running total per slot plus a queue of batch
records ``(timestamp, slots, counts)`` at request (batch) granularity -- every match of one
request carries the same instant, which is what the reference's per-match timestamps amount to
within one request. ``carry`` / ``record_counts`` cost O(ids touched), not a Python loop over
the whole library per request. The device pipeline turns the order dependency into a segmented
exclusive scan: for the k-th match of id X in a batch, ``count_before = carry[X] + k`` with
``carry[X]`` = matches of X still inside the window.

Extras over the reference: statistics / reset APIs exposed to the
admin endpoints, optional snapshot/restore to a JSON file (off by default, like the reference).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from collections import deque
from typing import Callable, Dict, Iterable, List, Optional

import numpy as np

log = logging.getLogger("log_parser_amd.frequency")


class FrequencyState:
    def __init__(self, window_hours: int = 1, clock: Callable[[], float] = time.time):
        self.window_s = float(window_hours) * 3600.0
        self.window_hours = window_hours
        self.clock = clock
        self._slot: Dict[str, int] = {}           # id -> slot (ids ever recorded or queried)
        self._names: List[str] = []
        self._seen = np.zeros(0, bool)            # slot recorded at least once (reference: map entry exists)
        self._tot = np.zeros(0, np.int64)         # matches inside the window per slot
        self._q: deque = deque()                  # (t, slots int64[], counts int64[]) per batch
        self._ids_cache = (None, None)
        self._lock = threading.RLock()

    # ---- slots
    def _slots(self, ids: List[str]) -> np.ndarray:
        obj, sl = self._ids_cache
        if obj is ids and sl is not None and sl.size == len(ids):
            return sl
        sl = np.fromiter((self._slot_of(p) for p in ids), np.int64, count=len(ids))
        self._ids_cache = (ids, sl)
        return sl

    def _slot_of(self, pid: str) -> int:
        s = self._slot.get(pid)
        if s is None:
            s = self._slot[pid] = len(self._names)
            self._names.append(pid)
            if s >= self._tot.size:
                grow = max(64, self._tot.size)
                self._tot = np.concatenate([self._tot, np.zeros(grow, np.int64)])
                self._seen = np.concatenate([self._seen, np.zeros(grow, bool)])
        return s

    def _prune(self, now: float) -> None:
        horizon = now - self.window_s
        q = self._q
        while q and q[0][0] <= horizon:
            _, sl, c = q.popleft()
            np.subtract.at(self._tot, sl, c)

    # ---- device pipeline interface
    def carry(self, ids: List[str]) -> np.ndarray:
        """Matches inside the window for each id (the exclusive-scan carry)."""
        now = self.clock()
        with self._lock:
            sl = self._slots(ids)
            self._prune(now)
            return self._tot[sl].copy()

    def record_counts(self, ids: List[str], counts: Iterable[int], now: Optional[float] = None) -> None:
        now = self.clock() if now is None else now
        c = np.asarray(counts if not isinstance(counts, (list, tuple)) else np.array(counts), np.int64).reshape(-1)
        c = c[:len(ids)]
        nz = np.flatnonzero(c > 0)
        if nz.size == 0:
            return
        with self._lock:
            sl = self._slots(ids)[nz]
            cc = c[nz].copy()
            np.add.at(self._tot, sl, cc)
            self._seen[sl] = True
            self._q.append((now, sl, cc))

    # ---- reference API surface (FrequencyTrackingService.java:101-161)
    def get_pattern_frequency(self, pid: str) -> Optional[dict]:
        with self._lock:
            s = self._slot.get(pid)
            if s is None or not self._seen[s]:
                return None
            self._prune(self.clock())
            c = int(self._tot[s])
            return {"patternId": pid, "currentCount": c, "hourlyRate": c / float(self.window_hours)}

    def statistics(self) -> Dict[str, int]:
        with self._lock:
            self._prune(self.clock())
            return {self._names[s]: int(self._tot[s]) for s in np.flatnonzero(self._seen[:len(self._names)])}

    def reset(self, pid: str) -> None:
        with self._lock:
            s = self._slot.get(pid)
            if s is None:
                return
            self._tot[s] = 0
            for _, sl, c in self._q:              # queued records of this id no longer count
                c[sl == s] = 0

    def reset_all(self) -> None:
        with self._lock:
            self._q.clear()
            self._tot[:] = 0
            self._seen[:] = False

    # ---- in-memory capture / rollback (elastic DP re-runs a step after a rank failure)
    def capture(self) -> dict:
        with self._lock:
            return {"q": [(t, sl.copy(), c.copy()) for t, sl, c in self._q], "tot": self._tot.copy(),
                    "seen": self._seen.copy(), "n": len(self._names)}

    def rollback(self, state: dict) -> None:
        with self._lock:
            self._q = deque((t, sl.copy(), c.copy()) for t, sl, c in state["q"])
            tot = np.zeros_like(self._tot)
            seen = np.zeros_like(self._seen)
            tot[:state["tot"].size] = state["tot"]
            seen[:state["seen"].size] = state["seen"]
            self._tot, self._seen = tot, seen

    # ---- checkpoint / resume: {"records": {id: [[t, count], ...]}}
    def _records(self) -> Dict[str, list]:
        rec: Dict[str, list] = {self._names[s]: [] for s in np.flatnonzero(self._seen[:len(self._names)])}
        for t, sl, c in self._q:
            for s, k in zip(sl.tolist(), c.tolist()):
                if k > 0:
                    rec[self._names[s]].append([t, k])
        return rec

    def snapshot(self, path: str) -> None:
        with self._lock:
            data = {"window_hours": self.window_hours, "records": self._records()}
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, path)

    def restore(self, path: str) -> None:
        if not os.path.exists(path):
            return
        with open(path) as f:
            data = json.load(f)
        with self._lock:
            self.reset_all()
            ev = []
            for k, v in data.get("records", {}).items():
                s = self._slot_of(k)
                self._seen[s] = True
                ev += [(float(t), s, int(c)) for t, c in v]
            for t, s, c in sorted(ev):
                sl = np.array([s], np.int64)
                cc = np.array([c], np.int64)
                self._tot[s] += c
                self._q.append((t, sl, cc))


class DeviceFrequencyState:
    """The same sliding-window state, resident in HBM next to the score kernel (SURVEY §2.5 K8,
    csrc/kernels/freq_state.hip): in-window totals per frequency key + a FIFO ring of
    (timestamp, key, count) batch records. ``carry_tensor`` evicts (kernel) and returns the totals
    as the score kernel's carry; ``record_tensor`` appends a batch's per-key counts (kernel).
    Neither touches the host: the only host input is the clock scalar. The admin / snapshot API
    reads the state back on demand. Keyed by one library's frequency ids (``ids``); one engine
    (GPU) owns it -- engines serving concurrently share a host ``FrequencyState`` instead.

    Works on CPU tensors too (the kernels' host twins), which is how the CPU tests pin it to
    ``golden.FrequencyTracker``."""

    device_resident = True

    def __init__(self, ids: List[str], window_hours: int, device, clock: Callable[[], float] = time.time,
                 capacity: int = 1 << 20):
        import torch
        self.ids = list(ids)
        self.window_hours = window_hours
        self.window_s = float(window_hours) * 3600.0
        self.clock = clock
        self.device = torch.device(device)
        K = max(len(self.ids), 1)
        self.tot = torch.zeros(K, dtype=torch.int64, device=self.device)
        self.seen = torch.zeros(K, dtype=torch.uint8, device=self.device)
        self.ht = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._alloc(max(int(capacity), 2 * K))
        self._tail_bound = 0          # host upper bound of ht[1] (no sync per batch)
        self._head_known = 0          # host lower bound of ht[0]
        self._last_now = float("-inf")
        self._lock = threading.RLock()
        self._index = {pid: i for i, pid in enumerate(self.ids)}

    # ---- storage
    def _alloc(self, cap: int) -> None:
        import torch
        self.cap = int(cap)
        self.t = torch.zeros(self.cap, dtype=torch.float64, device=self.device)
        self.key = torch.zeros(self.cap, dtype=torch.int32, device=self.device)
        self.cnt = torch.zeros(self.cap, dtype=torch.int32, device=self.device)

    def _ring(self) -> tuple:
        return (self.t.data_ptr(), self.key.data_ptr(), self.cnt.data_ptr(), self.cap, self.ht.data_ptr(),
                self.tot.data_ptr(), self.seen.data_ptr())

    def _stream(self) -> int:
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0

    def _records(self):
        """(t, key, cnt) host arrays of the live records, oldest first (syncs)."""
        h, tl = (int(x) for x in self.ht.cpu())
        if tl == h:
            return np.zeros(0), np.zeros(0, np.int64), np.zeros(0, np.int64)
        idx = (np.arange(h, tl) % self.cap)
        return (self.t.cpu().numpy()[idx], self.key.cpu().numpy()[idx].astype(np.int64),
                self.cnt.cpu().numpy()[idx].astype(np.int64))

    def _ensure_room(self, k: int, quiesce: Optional[Callable[[], None]] = None) -> None:
        """Keep at least ``k`` free ring slots; reads head/tail back only when the host bound says
        the ring may be full, and grows it (records kept in order) when it really is.
        ``quiesce``: with several engines sharing the window, waits until every earlier batch's
        window section has completed, so head / tail are exact and no kernel uses the old ring."""
        if self._tail_bound + k - self._head_known <= self.cap:
            return
        if quiesce is not None:
            quiesce()
        h, tl = (int(x) for x in self.ht.cpu())
        self._head_known, self._tail_bound = h, tl
        if tl + k - h <= self.cap:
            return
        import torch
        t, key, cnt = self._records()
        n = t.size
        self._alloc(max(2 * self.cap, n + 2 * k))
        if n:
            self.t[:n] = torch.from_numpy(t).to(self.device)
            self.key[:n] = torch.from_numpy(key.astype(np.int32)).to(self.device)
            self.cnt[:n] = torch.from_numpy(cnt.astype(np.int32)).to(self.device)
        self.ht.copy_(torch.tensor([0, n], dtype=torch.int64))
        self._head_known, self._tail_bound = 0, n

    def _now(self, now: Optional[float] = None) -> float:
        now = self.clock() if now is None else float(now)
        self._last_now = max(self._last_now, now)      # ring timestamps must not go backwards
        return self._last_now

    # ---- device pipeline interface
    def carry_tensor(self, now: Optional[float] = None):
        """Evict records at or before now - window; returns the in-window totals (device int64[K])."""
        from .native import N
        with self._lock:
            N.freq_evict(self._ring(), self._now(now) - self.window_s, self._stream(), self.device.type == "cuda")
            return self.tot

    def record_tensor(self, counts, now: Optional[float] = None, veto=None, gate=None) -> None:
        """Append this batch's per-key counts (int64 tensor on the state's device, >= K entries).
        ``veto`` (device int64[1], optional): nothing is recorded when it is non-zero (a DP step
        whose buffers overflowed and that re-runs). ``gate`` = (device counters int64[>=5], (gram,
        cand, ver, events) capacities): nothing is recorded when a counter exceeds its capacity."""
        from .native import N
        K = len(self.ids)
        if K == 0:
            return
        c = counts.to(device=self.device, dtype=__import__("torch").int64)
        with self._lock:
            self._ensure_room(K)
            N.freq_record(c.data_ptr(), K, self._now(now), self._ring(), self._stream(), self.device.type == "cuda",
                          veto.data_ptr() if veto is not None else 0,
                          gate[0].data_ptr() if gate is not None else 0, tuple(gate[1]) if gate is not None else ())
            self._tail_bound += K

    # host-array compatibility with FrequencyState (CPU callers, tests)
    def carry(self, ids: List[str]) -> np.ndarray:
        assert list(ids) == self.ids, "a device frequency state serves one library"
        return self.carry_tensor().cpu().numpy()[:len(ids)].copy()

    def record_counts(self, ids: List[str], counts: Iterable[int], now: Optional[float] = None) -> None:
        import torch
        assert list(ids) == self.ids, "a device frequency state serves one library"
        c = torch.as_tensor(np.asarray(counts, np.int64).reshape(-1)[:len(ids)])
        self.record_tensor(c, now)

    # ---- reference API surface (FrequencyTrackingService.java:101-161)
    def _pruned_totals(self):
        self.carry_tensor()
        return self.tot.cpu().numpy(), self.seen.cpu().numpy()

    def get_pattern_frequency(self, pid: str) -> Optional[dict]:
        with self._lock:
            k = self._index.get(pid)
            if k is None:
                return None
            tot, seen = self._pruned_totals()
            if not seen[k]:
                return None
            c = int(tot[k])
            return {"patternId": pid, "currentCount": c, "hourlyRate": c / float(self.window_hours)}

    def statistics(self) -> Dict[str, int]:
        with self._lock:
            tot, seen = self._pruned_totals()
            return {self.ids[k]: int(tot[k]) for k in np.flatnonzero(seen[:len(self.ids)])}

    def reset(self, pid: str) -> None:
        with self._lock:
            k = self._index.get(pid)
            if k is None:
                return
            self.tot[k] = 0
            self.cnt.masked_fill_(self.key == k, 0)           # queued records no longer count

    def reset_all(self) -> None:
        with self._lock:
            self.tot.zero_()
            self.seen.zero_()
            self.ht.zero_()
            self._head_known = self._tail_bound = 0

    # ---- capture / rollback (elastic DP re-runs a step after a rank failure)
    def capture(self) -> dict:
        with self._lock:
            # the whole ring is cloned: records appended after the capture may reuse slots that
            # were live at capture time, and rollback must restore their timestamps and keys too
            return {"ht": self.ht.clone(), "tot": self.tot.clone(), "seen": self.seen.clone(),
                    "t": self.t.clone(), "key": self.key.clone(), "cnt": self.cnt.clone()}

    def rollback(self, state: dict) -> None:
        with self._lock:
            self.t, self.key, self.cap = state["t"].clone(), state["key"].clone(), state["t"].numel()
            self.cnt = state["cnt"].clone()
            self.ht.copy_(state["ht"])
            self.tot.copy_(state["tot"])
            self.seen.copy_(state["seen"])
            h, tl = (int(x) for x in self.ht.cpu())
            self._head_known, self._tail_bound = h, tl

    def to_host_state(self) -> "FrequencyState":
        """A host ``FrequencyState`` holding the same in-window records (the CPU fallback's copy
        of the window after a device fault); empty when the device cannot be read."""
        fs = FrequencyState(self.window_hours, clock=self.clock)
        try:
            with self._lock:
                t, key, cnt = self._records()
                seen = self.seen.cpu().numpy()
        except Exception:  # noqa: BLE001 - a failed device: start from an empty window
            log.warning("device frequency window unreadable; the CPU fallback starts from an empty window")
            return fs
        for k in np.flatnonzero(seen[:len(self.ids)]):
            slot = fs._slot_of(self.ids[k])       # (may grow fs._seen: index it afterwards)
            fs._seen[slot] = True
        for a, k, c in zip(t.tolist(), key.tolist(), cnt.tolist()):
            if c > 0:
                s = fs._slot_of(self.ids[k])
                fs._tot[s] += c
                fs._q.append((float(a), np.array([s], np.int64), np.array([c], np.int64)))
        return fs

    # ---- checkpoint / resume: the same JSON as FrequencyState
    def snapshot(self, path: str) -> None:
        with self._lock:
            t, key, cnt = self._records()
            seen = self.seen.cpu().numpy()
            rec: Dict[str, list] = {self.ids[k]: [] for k in np.flatnonzero(seen[:len(self.ids)])}
            for a, k, c in zip(t.tolist(), key.tolist(), cnt.tolist()):
                if c > 0:
                    rec[self.ids[k]].append([a, c])
            data = {"window_hours": self.window_hours, "records": rec}
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, path)

    def restore(self, path: str) -> None:
        import torch
        if not os.path.exists(path):
            return
        with open(path) as f:
            data = json.load(f)
        with self._lock:
            self.reset_all()
            ev = []
            for pid, v in data.get("records", {}).items():
                k = self._index.get(pid)
                if k is None:
                    continue
                self.seen[k] = 1
                ev += [(float(a), k, int(c)) for a, c in v]
            ev.sort()
            n = len(ev)
            self._ensure_room(n + 1)
            if n:
                self.t[:n] = torch.tensor([e[0] for e in ev], dtype=torch.float64)
                self.key[:n] = torch.tensor([e[1] for e in ev], dtype=torch.int32)
                self.cnt[:n] = torch.tensor([e[2] for e in ev], dtype=torch.int32)
                tot = np.zeros(self.tot.numel(), np.int64)
                np.add.at(tot, [e[1] for e in ev], [e[2] for e in ev])
                self.tot.copy_(torch.from_numpy(tot))
                self._last_now = max(self._last_now, ev[-1][0])
            self.ht.copy_(torch.tensor([0, n], dtype=torch.int64))
            self._head_known, self._tail_bound = 0, n


class MirroredFrequencyState(FrequencyState):
    """Host copy of a device-resident window for the CPU fallback after a device failure
    (availability only): reads come from the copy; records go to the copy and, best
    effort, to the device window, so a recovered GPU keeps counting the fallback's matches."""

    def __init__(self, dev: DeviceFrequencyState):
        host = dev.to_host_state()
        super().__init__(dev.window_hours, clock=dev.clock)
        self._slot, self._names, self._seen, self._tot, self._q = \
            host._slot, host._names, host._seen, host._tot, host._q
        self._dev = dev

    def record_counts(self, ids: List[str], counts: Iterable[int], now: Optional[float] = None) -> None:
        now = self.clock() if now is None else now
        super().record_counts(ids, counts, now)
        try:
            self._dev.record_counts(ids, counts, now)
        except Exception:  # noqa: BLE001 - the device may be the thing that failed
            log.warning("could not record the fallback batch in the device frequency window")


class SharedFrequencyState(DeviceFrequencyState):
    """ONE window shared by the serving PROCESSES of a node (one process per GPU,
    ``serve/procs.py``) -- the reference's single process-global window
    (FrequencyTrackingService.java:25) kept across processes instead of across threads.

    The window lives in HOST shared memory (``N.SharedWindow``, csrc/runtime/proc_shared.h): a ring
    of (timestamp, key, count) records, in-window totals and seen flags per key, one block per
    generation (a grown ring is a new block; the others re-map it at their next access). Whatever
    GPU a process drives, its native request runner evicts, copies the carry and records on the host
    inside the batch's window section, and its score kernel reads the carry from pinned memory
    (``RequestRunner.run(hw=...)``): no GPU memory crosses processes, no peer access, and every
    worker keeps the native runner. The section is entered with an arrival ticket drawn once the
    batch's matching is DONE, so it holds no other process's matching.

    CPU engines (and the Python paths of GPU engines) use the same window through the
    ``DeviceFrequencyState`` API on host views of the shared arrays. The admin / snapshot API takes
    its own ticket and runs between batches."""

    device_resident = False          # host memory: GPU engines reach it through the runner's host window

    def __init__(self, ids: List[str], window_hours: int, shared, clock: Callable[[], float] = time.time,
                 capacity: int = 1 << 20, create: bool = False):
        import torch
        from .native import N
        self.ids = list(ids)
        self.window_hours = window_hours
        self.window_s = float(window_hours) * 3600.0
        self.clock = clock
        self.device = torch.device("cpu")
        self.sh = shared
        self._K = max(len(self.ids), 1)
        self._lock = threading.RLock()
        self._index = {pid: i for i, pid in enumerate(self.ids)}
        self._tls = threading.local()
        self._views: tuple = ()
        self._base = 0
        self._head_known = self._tail_bound = 0       # (DeviceFrequencyState bookkeeping: unused here)
        if create:
            seq = self.sh.take()                      # the first ticket: nothing runs before the window
            try:
                self.sh.host.wait(seq)
                self.sh.dev.wait(seq)
                self.win = N.SharedWindow(shared, self._K, self.window_s, True, max(int(capacity), 2 * self._K))
            finally:
                self.sh.host.done(seq)
                self.sh.dev.done(seq)
        else:
            if int(self.sh.generation) == 0:
                raise RuntimeError("the shared frequency window has not been created yet")
            if int(self.sh.nkeys) != self._K:
                raise RuntimeError(f"shared window has {self.sh.nkeys} keys, this library {self._K}")
            self.win = N.SharedWindow(shared, self._K, self.window_s, False)

    # ---- host views of the current generation
    def _current(self) -> tuple:
        import torch
        from .native import N
        a = self.win.arrays()                         # re-maps after a growth
        if a[0] != self._base:
            cap, K = int(a[6]), self._K
            spec = [("float64", cap), ("int32", cap), ("int32", cap), ("int64", 2), ("int64", K), ("uint8", K)]
            self._views = tuple(torch.from_dlpack(N.dlpack(int(ptr), n, dt, -1)) for ptr, (dt, n) in zip(a[:6], spec))
            self._base = a[0]
        return self._views

    t = property(lambda s: s._current()[0])
    key = property(lambda s: s._current()[1])
    cnt = property(lambda s: s._current()[2])
    ht = property(lambda s: s._current()[3])
    tot = property(lambda s: s._current()[4])
    seen = property(lambda s: s._current()[5])

    @property
    def cap(self) -> int:
        return int(self.win.arrays()[6])

    _last_now = property(lambda s: s.sh.last_now, lambda s, v: s.win.now(float(v)))

    def _alloc(self, cap: int) -> None:
        raise NotImplementedError("the shared window grows in N.SharedWindow.ensure_room")

    def _ensure_room(self, k: int, quiesce: Optional[Callable[[], None]] = None) -> None:
        self.win.ensure_room(int(k))

    def _now(self, now: Optional[float] = None) -> float:
        return self.win.now(self.clock() if now is None else float(now))

    # ---- the window section's steps (the caller holds the turns)
    def carry_tensor(self, now: Optional[float] = None):
        with self._lock:
            self.win.evict(self._now(now) - self.window_s)
            return self.tot

    def record_tensor(self, counts, now: Optional[float] = None, veto=None, gate=None) -> None:
        import torch
        K = len(self.ids)
        if K == 0 or (veto is not None and int(veto.item())):
            return
        if gate is not None:             # (DeviceFrequencyState.record_tensor's gate, read here)
            g, k, v, _, ne = gate[0][:5].tolist()
            if g > gate[1][0] or k > gate[1][1] or v > gate[1][2] or ne > gate[1][3]:
                return
        c = counts.to(device="cpu", dtype=torch.int64).contiguous()
        if c.numel() < K:
            c = torch.cat([c, torch.zeros(K - c.numel(), dtype=torch.int64)])
        with self._lock:
            self.win.record(c.data_ptr(), K, self._now(now))

    # ---- the admin API runs between batches, under an arrival ticket of its own
    def _exclusive_enter(self) -> None:
        d = getattr(self._tls, "depth", 0)
        self._tls.depth = d + 1
        if d:
            return
        self._tls.seq = self.win.enter()

    def _exclusive_exit(self) -> None:
        self._tls.depth -= 1
        if self._tls.depth:
            return
        self.win.leave(self._tls.seq)

    def _exclusive(self, fn, *a):
        self._exclusive_enter()
        try:
            return fn(*a)
        finally:
            self._exclusive_exit()

    def get_pattern_frequency(self, pid: str) -> Optional[dict]:
        return self._exclusive(super().get_pattern_frequency, pid)

    def statistics(self) -> Dict[str, int]:
        return self._exclusive(super().statistics)

    def reset(self, pid: str) -> None:
        self._exclusive(super().reset, pid)

    def reset_all(self) -> None:
        self._exclusive(super().reset_all)

    def snapshot(self, path: str) -> None:
        self._exclusive(super().snapshot, path)

    def restore(self, path: str) -> None:
        self._exclusive(super().restore, path)

    def capture(self) -> dict:
        raise NotImplementedError("the elastic DP capture / rollback does not apply to a shared serving window")

    rollback = capture
