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

* the window lives in host shared memory (``SharedFrequencyState`` over ``N.SharedWindow``),
  created by the first worker; every worker's native request runner evicts, copies the carry and
  records on the host inside its batch's window section, and its score kernel reads the pinned
  carry -- so the runner serves on every GPU, with no IPC of GPU memory and no peer access;
* a batch draws its arrival ticket once its MATCHING IS DONE (inside the runner, after the events,
  context features and ranks have finished on its GPU); its window section (eviction, score with
  the in-window carry, record) runs after every earlier ticket's, whichever process holds them
  (cross-process turns on a futex). Matching overlaps freely across processes and GPUs.

So requests sent one after another get exactly the responses one process gives, and concurrent
ones the responses of SOME arrival order, as in the reference.

Failures: a worker that dies holding a ticket has it released by the others once they find its pid
gone (``ProcTurn::wait``), and the SURVIVORS KEEP SERVING (SO_REUSEPORT sends new connections to the
live listeners). The supervisor restarts a dead worker on the same device (``server.max-restarts``
per worker; the restarted process attaches to the existing window) and stops the group only when a
worker has exhausted its restarts or exits during start-up. A record the dead worker had half
applied stays as it is -- as a reference request thread that dies mid-request leaves the
``recordPatternMatch`` calls it already made (ScoringService.java:84-88, per match).
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

ENV_SHM, ENV_WORKER, ENV_NPROC = "LP_SERVE_SHM", "LP_SERVE_WORKER", "LP_SERVE_NPROC"


class WorkerContext:
    """This process's place in a serving group (built from the supervisor's environment)."""

    def __init__(self, shared, index: int, nproc: int):
        self.shared = shared
        self.index = index
        self.nproc = nproc
        # the first worker creates the window; a restarted one (generation > 0) attaches to it
        self.owner = index == 0 and int(shared.generation) == 0

    @staticmethod
    def from_env() -> Optional["WorkerContext"]:
        name = os.environ.get(ENV_SHM)
        if not name:
            return None
        from ..native import N
        return WorkerContext(N.ProcShared(name, False), int(os.environ[ENV_WORKER]), int(os.environ[ENV_NPROC]))

    def frequency_state(self, lib, cfg: Config):
        """The shared window: created by the first worker (after which it restores a snapshot, if
        configured), attached by the others once it exists."""
        from ..frequency import SharedFrequencyState
        hours = cfg.scoring.freq_window_hours
        if self.owner:
            return SharedFrequencyState(lib.freq_ids, hours, self.shared, create=True)
        deadline = time.monotonic() + 600
        while not self.shared.up(0) or int(self.shared.generation) == 0:
            if time.monotonic() > deadline:
                raise RuntimeError("serving worker 0 never created the shared frequency window")
            time.sleep(0.01)
        return SharedFrequencyState(lib.freq_ids, hours, self.shared, create=False)

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


def _worker_argv(argv: Sequence[str], device: str) -> List[str]:
    keep = [a for a in argv if not a.startswith(("-Dserver.processes=", "-Dengine.device=",
                                                  "-Dengine.serve-devices="))]
    return ["-m", "log_parser_amd.serve"] + keep + ["-Dserver.processes=1", f"-Dengine.device={device}",
                                                    "-Dengine.serve-devices="]


def run_processes(argv: Sequence[str], cfg: Config, n: int, stop=None, ready_timeout_s: float = 900.0) -> int:
    """Supervisor: the shared segment, ``n`` workers (restarted when they die), their exit status.
    ``stop`` (an Event): set to stop the group (signals set it in ``serve.__main__``)."""
    from ..native import N
    name = f"/lp-serve-{os.getpid()}-{int(time.time() * 1e3) % 100000}"
    shared = N.ProcShared(name, True, n)
    procs: List[subprocess.Popen] = []
    devs = worker_devices(cfg, n)
    max_restarts = int(cfg.get("server.max-restarts", 3) or 0)
    restarts = [0] * n
    log.info("%d serving processes on %s, one host frequency window", n, devs)

    def spawn(i: int) -> subprocess.Popen:
        env = dict(os.environ)
        env.update({ENV_SHM: name, ENV_WORKER: str(i), ENV_NPROC: str(n)})
        return subprocess.Popen([sys.executable] + _worker_argv(argv, devs[i]), env=env)
    try:
        for i in range(n):
            procs.append(spawn(i))
        t0, announced = time.monotonic(), False
        while True:
            codes = [p.poll() for p in procs]
            if all(c == 0 for c in codes):
                return 0
            for i, c in enumerate(codes):
                if c in (None, 0):
                    continue
                if not announced or restarts[i] >= max_restarts:
                    log.error("serving worker %d exited with status %s (%s): stopping the group", i, c,
                              "during start-up" if not announced else f"after {restarts[i]} restarts")
                    return c
                restarts[i] += 1
                shared.restarts = int(shared.restarts) + 1
                log.error("serving worker %d exited with status %s: restarting it (%d/%d); the others keep serving",
                          i, c, restarts[i], max_restarts)
                procs[i] = spawn(i)
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
