"""Prometheus-text metrics for the service (the reference exports none)."""
from __future__ import annotations

import threading
from typing import Dict

_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


class _Hist:
    def __init__(self):
        self.counts = [0] * (len(_BUCKETS) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float):
        self.sum += v
        self.n += 1
        for i, b in enumerate(_BUCKETS):
            if v <= b:
                self.counts[i] += 1
                return
        self.counts[-1] += 1

    def render(self, name: str, out: list):
        c = 0
        for i, b in enumerate(_BUCKETS):
            c += self.counts[i]
            out.append(f'{name}_bucket{{le="{b}"}} {c}')
        c += self.counts[-1]
        out.append(f'{name}_bucket{{le="+Inf"}} {c}')
        out.append(f"{name}_sum {self.sum}")
        out.append(f"{name}_count {self.n}")


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.requests: Dict[int, int] = {}
        self.bytes_total = 0
        self.latency = _Hist()
        self.batch_latency = _Hist()
        self.batches = 0
        self.batched_requests = 0
        self.device_failures = 0
        self.bt_exhausted = 0          # backtracker finds that hit the step budget (counted "no match")
        self.freq: Dict[str, int] = {}

    def observe_request(self, code: int, seconds: float, nbytes: int):
        with self._lock:
            self.requests[code] = self.requests.get(code, 0) + 1
            self.bytes_total += nbytes
            if code == 200:
                self.latency.observe(seconds)

    def observe_requests(self, code: int, seconds, nbytes: int):
        """Many requests of one status at once (the native front end's batch completion)."""
        with self._lock:
            self.requests[code] = self.requests.get(code, 0) + len(seconds)
            self.bytes_total += nbytes
            if code == 200:
                for s in seconds:
                    self.latency.observe(s)

    def observe_batch(self, n: int, seconds: float):
        with self._lock:
            self.batches += 1
            self.batched_requests += n
            self.batch_latency.observe(seconds)

    def set_frequency(self, stats: Dict[str, int]):
        with self._lock:
            self.freq = dict(stats)

    def render(self) -> str:
        with self._lock:
            out = ["# TYPE lp_requests_total counter"]
            for code, n in sorted(self.requests.items()):
                out.append(f'lp_requests_total{{code="{code}"}} {n}')
            out += ["# TYPE lp_log_bytes_total counter", f"lp_log_bytes_total {self.bytes_total}",
                    "# TYPE lp_request_seconds histogram"]
            self.latency.render("lp_request_seconds", out)
            out += ["# TYPE lp_batches_total counter", f"lp_batches_total {self.batches}",
                    "# TYPE lp_batched_requests_total counter", f"lp_batched_requests_total {self.batched_requests}",
                    "# TYPE lp_batch_seconds histogram"]
            self.batch_latency.render("lp_batch_seconds", out)
            out += ["# TYPE lp_device_failures_total counter", f"lp_device_failures_total {self.device_failures}",
                    "# TYPE lp_backtracker_budget_exhausted_total counter",
                    f"lp_backtracker_budget_exhausted_total {self.bt_exhausted}"]
            out.append("# TYPE lp_pattern_frequency gauge")
            for k, v in sorted(self.freq.items()):
                out.append(f'lp_pattern_frequency{{pattern_id="{k}"}} {v}')
            return "\n".join(out) + "\n"
