"""Persistent sliding-window frequency state (reference ``FrequencyTrackingService.java:20-162``).

The reference keeps a process-global ``ConcurrentHashMap<patternId, PatternFrequency>`` that
survives across requests (``FrequencyTrackingService.java:25``) and computes a pattern's
penalty from its hourly rate *before* recording the current match (``ScoringService.java:84-88``).

Here the state is a per-id deque of ``(timestamp, count)`` records at request (batch)
granularity — every match of one request carries the same instant, which is what the
reference's per-match timestamps amount to within one request. The device pipeline turns the
order dependency into a segmented exclusive scan: for the k-th match of id X in a batch,
``count_before = carry[X] + k`` with ``carry[X]`` = matches of X still inside the window.

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
        self._rec: Dict[str, deque] = {}
        self._tot: Dict[str, int] = {}
        self._lock = threading.RLock()

    def _prune(self, pid: str, now: float) -> None:
        dq = self._rec.get(pid)
        if not dq:
            return
        horizon = now - self.window_s
        while dq and dq[0][0] <= horizon:
            _, c = dq.popleft()
            self._tot[pid] -= c

    def carry(self, ids: List[str]) -> np.ndarray:
        """Matches inside the window for each id (the exclusive-scan carry)."""
        now = self.clock()
        out = np.zeros(len(ids), np.int64)
        with self._lock:
            for i, pid in enumerate(ids):
                if pid in self._rec:
                    self._prune(pid, now)
                    out[i] = self._tot[pid]
        return out

    def record_counts(self, ids: List[str], counts: Iterable[int], now: Optional[float] = None) -> None:
        now = self.clock() if now is None else now
        with self._lock:
            for pid, c in zip(ids, counts):
                c = int(c)
                if c <= 0:
                    continue
                if pid not in self._rec:
                    self._rec[pid] = deque()
                    self._tot[pid] = 0
                self._rec[pid].append((now, c))
                self._tot[pid] += c

    # ---- reference API surface (FrequencyTrackingService.java:101-161)
    def get_pattern_frequency(self, pid: str) -> Optional[dict]:
        with self._lock:
            if pid not in self._rec:
                return None
            self._prune(pid, self.clock())
            c = self._tot[pid]
            return {"patternId": pid, "currentCount": c, "hourlyRate": c / float(self.window_hours)}

    def statistics(self) -> Dict[str, int]:
        now = self.clock()
        with self._lock:
            for pid in list(self._rec):
                self._prune(pid, now)
            return dict(self._tot)

    def reset(self, pid: str) -> None:
        with self._lock:
            if pid in self._rec:
                self._rec[pid].clear()
                self._tot[pid] = 0

    def reset_all(self) -> None:
        with self._lock:
            self._rec.clear()
            self._tot.clear()

    # ---- in-memory capture / rollback (elastic DP re-runs a step after a rank failure)
    def capture(self) -> dict:
        with self._lock:
            return {k: list(v) for k, v in self._rec.items()}

    def rollback(self, state: dict) -> None:
        with self._lock:
            self._rec = {k: deque(v) for k, v in state.items()}
            self._tot = {k: sum(c for _, c in v) for k, v in state.items()}

    # ---- checkpoint / resume
    def snapshot(self, path: str) -> None:
        with self._lock:
            data = {"window_hours": self.window_hours,
                    "records": {k: list(map(list, v)) for k, v in self._rec.items()}}
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
            self._rec.clear()
            self._tot.clear()
            for k, v in data.get("records", {}).items():
                self._rec[k] = deque((float(t), int(c)) for t, c in v)
                self._tot[k] = sum(int(c) for _, c in v)
