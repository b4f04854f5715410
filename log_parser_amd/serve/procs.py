"""Node-scale serving: one serving PROCESS per GPU, sharing one frequency window.

``python -m log_parser_amd.serve -Dserver.processes=N`` (or -1: one per visible GPU) makes the
launching process a supervisor that never touches the GPU (like ``utils/launch.py`` for ranks): it
creates the shared segment (``N.ProcShared``, csrc/runtime/proc_shared.h) and starts N fresh
interpreters. Each worker is a complete single-engine server -- its own native HTTP listeners on
the SAME port (SO_REUSEPORT: the kernel spreads connections over the processes), its own GIL, pump
thread and pack / device / emit pipeline, its own GPU (``engine.serve-devices[i % n]``, or
``engine.device`` for all of them: the one-GPU rehearsal). What they share is what the reference
shares between its request threads: ONE sliding frequency window (FrequencyTrackingService.java:25
one map, :41-56 record) with penalty-before-record in arrival order (ScoringService.java:84-88):

* worker 0 allocates the window in its GPU's HBM and publishes an IPC handle
  (``hipIpcGetMemHandle``); the others map it (``hipIpcOpenMemHandle``) -- ``SharedFrequencyState``;
* a batch draws an arrival ticket from the segment when it enters its device stage; its window
  section (eviction, score with the in-window carry, record) runs after every earlier ticket's,
  whichever process holds them (``ProcessWindowTurn``: cross-process turns on a futex). Matching
  runs before the turn, concurrently on every process.

So requests sent one after another get exactly the responses one process gives, and concurrent
ones the responses of SOME arrival order, as in the reference. A worker that dies releases nothing
by itself: the others release its tickets after they find its pid gone (ProcTurn::wait), and the
supervisor stops the whole group with the first failing worker's status.
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional, Sequence

from ..utils.config import Config

log = logging.getLogger("log_parser_amd.server")

ENV_SHM, ENV_WORKER, ENV_NPROC, ENV_WINDOW = "LP_SERVE_SHM", "LP_SERVE_WORKER", "LP_SERVE_NPROC", "LP_SERVE_WINDOW"


class WorkerContext:
    """This process's place in a serving group (built from the supervisor's environment)."""

    def __init__(self, shared, index: int, nproc: int, window: str = "device"):
        self.shared = shared
        self.index = index
        self.nproc = nproc
        self.owner = index == 0
        self.window = window            # "device" or "host" (decided by the supervisor for all)

    @staticmethod
    def from_env() -> Optional["WorkerContext"]:
        name = os.environ.get(ENV_SHM)
        if not name:
            return None
        from ..native import N
        return WorkerContext(N.ProcShared(name, False), int(os.environ[ENV_WORKER]), int(os.environ[ENV_NPROC]),
                             os.environ.get(ENV_WINDOW, "device"))

    def frequency_state(self, lib, cfg: Config):
        """The shared window: created by worker 0 (on its device), mapped by the others once
        worker 0 reports it ready (after a snapshot restore, if any)."""
        import torch
        from ..engine import resolve_device
        from ..frequency import SharedFrequencyState
        dev = resolve_device(str(cfg["engine.device"]))
        hours = cfg.scoring.freq_window_hours
        host = self.window == "host" or dev.type != "cuda"
        wdev = torch.device("cpu") if host else dev
        if self.owner:
            st = SharedFrequencyState(lib.freq_ids, hours, wdev, self.shared, create=True)
            return self._placed(st, host, dev)
        deadline = time.monotonic() + 600
        while not self.shared.up(0):
            if time.monotonic() > deadline:
                raise RuntimeError("serving worker 0 never created the shared frequency window")
            time.sleep(0.01)
        if not host:
            from ..native import N
            me = dev.index if dev.index is not None else torch.cuda.current_device()
            if me != self.shared.home_device and not N.enable_peer_access(me, self.shared.home_device):
                raise RuntimeError(f"no peer access from {dev} to the window's GPU {self.shared.home_device}")
        return self._placed(SharedFrequencyState(lib.freq_ids, hours, wdev, self.shared, create=False), host, dev)

    @staticmethod
    def _placed(st, host: bool, dev):
        if host and dev.type == "cuda":
            # a GPU engine over the host window: it reads the carry and records counts through the
            # host (Engine.freq_on_device False), as with an engine-private host FrequencyState
            st.device_resident = False
        return st

    def window_ready(self) -> None:
        self.shared.mark_up(self.index, os.getpid())


def process_count(cfg: Config) -> int:
    n = int(cfg.get("server.processes", 1) or 1)
    if n >= 0:
        return max(n, 1)
    import torch                       # device_count() does not initialise the GPU on this image
    return max(torch.cuda.device_count(), 1)


def worker_devices(cfg: Config, n: int) -> List[str]:
    spec = str(cfg.get("engine.serve-devices", "") or "").strip()
    if spec == "all":
        import torch
        devs = [f"cuda:{i}" for i in range(torch.cuda.device_count())]
    else:
        devs = [x.strip() for x in spec.split(",") if x.strip()]
    devs = devs or [str(cfg["engine.device"])]
    return [devs[i % len(devs)] for i in range(n)]


def window_placement(cfg: Config, devs: Sequence[str]) -> str:
    """``server.window``: "device" / "host", or auto -- device when every worker is on one GPU or
    ``engine.serve.peer-window`` is on (workers on other GPUs then map worker 0's HBM over xGMI, a
    path no multi-GPU run has pinned yet), else host."""
    w = str(cfg.get("server.window", "auto") or "auto")
    if w in ("device", "host"):
        return w
    if len(set(devs)) <= 1 or bool(cfg.get("engine.serve.peer-window", False)):
        return "device"
    return "host"


def _worker_argv(argv: Sequence[str], device: str) -> List[str]:
    keep = [a for a in argv if not a.startswith(("-Dserver.processes=", "-Dengine.device=",
                                                  "-Dengine.serve-devices="))]
    return ["-m", "log_parser_amd.serve"] + keep + ["-Dserver.processes=1", f"-Dengine.device={device}",
                                                    "-Dengine.serve-devices="]


def run_processes(argv: Sequence[str], cfg: Config, n: int, stop=None, ready_timeout_s: float = 900.0) -> int:
    """Supervisor: the shared segment, ``n`` workers, their exit status. ``stop`` (an Event):
    set to stop the group (signals set it in ``serve.__main__``)."""
    from ..native import N
    name = f"/lp-serve-{os.getpid()}-{int(time.time() * 1e3) % 100000}"
    shared = N.ProcShared(name, True, n)
    procs: List[subprocess.Popen] = []
    devs = worker_devices(cfg, n)
    window = window_placement(cfg, devs)
    log.info("%d serving processes on %s, %s frequency window", n, devs, window)
    try:
        for i, dev in enumerate(devs):
            env = dict(os.environ)
            env.update({ENV_SHM: name, ENV_WORKER: str(i), ENV_NPROC: str(n), ENV_WINDOW: window})
            procs.append(subprocess.Popen([sys.executable] + _worker_argv(argv, dev), env=env))
        t0, announced = time.monotonic(), False
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                log.error("a serving worker exited with status %s: stopping the group", bad[0])
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            if not announced and all(shared.up(i) for i in range(n)):
                announced = True
                log.info("%d serving processes up (%.1f s)", n, time.monotonic() - t0)
            elif not announced and time.monotonic() - t0 > ready_timeout_s:
                log.error("serving workers not ready after %.0f s", ready_timeout_s)
                return 124
            if stop is not None and stop.wait(0.2):
                return 0
            if stop is None:
                time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        N.ProcShared.unlink(name, int(shared.generation))
