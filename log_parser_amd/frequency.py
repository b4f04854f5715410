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
import os
import threading
import time
from collections import deque
from typing import Callable, Dict, Iterable, List, Optional

import numpy as np


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
