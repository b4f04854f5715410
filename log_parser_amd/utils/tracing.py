"""Per-stage tracing (the reference only reports ``processingTimeMs``,
``AnalysisService.java:51,169``).

* Device stages are timed with HIP events recorded on the compute stream at stage boundaries:
  no host synchronisation is added -- the events are read once, after the batch's own final
  device->host copy. On CPU the same marks are ``perf_counter`` stamps.
* Host stages (D2H + JSON emission) are plain ``perf_counter`` intervals.
* :func:`torch_profile` wraps a region in ``torch.profiler`` (CPU + HIP activities) and writes a
  Chrome trace, for host-orchestration profiling next to ``rocprofv3`` kernel traces.

Enabled by ``engine.trace=true`` (stage timings are then added to the response metadata as
``stageTimingsMs`` and logged at DEBUG) or ``Engine.profile = True`` (bench ``--profile``).
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, Optional

import torch

_MARKS = "_marks"


def start(timings: dict, device: torch.device) -> None:
    """Anchor for the next device stage (a new anchor breaks the chain: host gaps between
    ``finish`` and the next ``start`` are not attributed to any stage)."""
    timings.setdefault(_MARKS, []).append((None, _stamp(device)))


def mark(timings: dict, name: str, device: torch.device) -> None:
    """End of stage ``name`` (started at the previous mark/anchor)."""
    timings.setdefault(_MARKS, []).append((name, _stamp(device)))


def _stamp(device: torch.device):
    if device.type == "cuda":
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(device))
        return ev
    return time.perf_counter()


def resolve(timings: dict) -> Dict[str, float]:
    """Milliseconds per stage (accumulated over repeats); synchronises on the last event only."""
    out = {k: v for k, v in timings.items() if k != _MARKS}
    marks = timings.get(_MARKS) or []
    if marks and isinstance(marks[-1][1], torch.cuda.Event):
        marks[-1][1].synchronize()
    for (_, a), (name, b) in zip(marks, marks[1:]):
        if name is None:
            continue
        if isinstance(a, torch.cuda.Event):
            ms = a.elapsed_time(b)
        else:
            ms = (b - a) * 1e3
        out[name] = out.get(name, 0.0) + ms
    return out


class HostTimer:
    """``with HostTimer(timings, "json"): ...`` adds a host-side interval when ``enabled``."""

    __slots__ = ("timings", "name", "enabled", "t0")

    def __init__(self, timings: Optional[dict], name: str):
        self.timings, self.name, self.enabled = timings, name, timings is not None

    def __enter__(self):
        if self.enabled:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            self.timings[self.name] = self.timings.get(self.name, 0.0) + (time.perf_counter() - self.t0) * 1e3
        return False


@contextlib.contextmanager
def torch_profile(path: str, device: Optional[torch.device] = None):
    """Chrome trace of the enclosed region (host ops + HIP kernels) written to ``path``."""
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU]
    if (device is None and torch.cuda.is_available()) or (device is not None and device.type == "cuda"):
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, record_shapes=False) as prof:
        yield prof
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    prof.export_chrome_trace(path)
