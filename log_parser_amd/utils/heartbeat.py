"""Per-rank phase heartbeats and a hang guard for multi-process jobs (the 8-GPU bench).

A first-ever world-8 RCCL run that hangs -- a rank stuck in ``init_process_group``, one that
never reaches a collective, a kernel that never finishes -- would otherwise burn the driver's whole
timeout and leave no trace of WHICH rank stalled WHERE. Every rank therefore writes its last
completed phase (``init_process_group``, ``warmup 2``, ``timed 7``, ...) to a small file in a
directory all ranks of the node share, and runs a watchdog thread: when NO rank has advanced for
``stall_s`` seconds (collectives couple the ranks, so a stuck rank stalls them all), or the job
exceeds ``total_s``, rank 0 prints ONE JSON line ``{"status": "timeout", "phases": {...}}`` on
stdout, every rank reports on stderr, and the ranks exit with status 124 -- no restart. The
launching parent (``utils/launch.spawn_local_ranks``) applies the same deadline from outside as a
backstop and prints the same diagnostic from the files if the ranks could not.

The directory is derived from the rendezvous (``MASTER_ADDR`` / ``MASTER_PORT``), so it works
under ``torch.distributed.run`` as well as under the bench's own launcher.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import threading
import time
from typing import Callable, Dict, Optional

ENV_DIR = "LP_HEARTBEAT_DIR"


def default_dir() -> str:
    """One directory per rendezvous on this node (every rank derives the same path)."""
    d = os.environ.get(ENV_DIR)
    if d:
        return d
    tag = f"{os.environ.get('MASTER_ADDR', 'local')}-{os.environ.get('MASTER_PORT', '0')}"
    return os.path.join(tempfile.gettempdir(), f"lp-heartbeat-{os.getuid()}-{tag}")


def read_phases(directory: str, world: int) -> Dict[str, dict]:
    """{rank: {"phase": ..., "age_s": seconds since it was written}} for every rank's file."""
    out: Dict[str, dict] = {}
    now = time.time()
    for r in range(world):
        p = os.path.join(directory, f"rank{r}")
        try:
            with open(p) as f:
                rec = json.load(f)
            out[str(r)] = {"phase": rec.get("phase"), "age_s": round(now - float(rec.get("t", now)), 1)}
        except (OSError, ValueError):
            out[str(r)] = {"phase": None, "age_s": None}
    return out


def last_progress(directory: str, world: int) -> float:
    """Wall time of the most recent heartbeat of any rank (0 if none yet)."""
    best = 0.0
    for r in range(world):
        try:
            best = max(best, os.stat(os.path.join(directory, f"rank{r}")).st_mtime)
        except OSError:
            pass
    return best


def timeout_record(metric: str, world: int, phases: Dict[str, dict], reason: str, waited_s: float) -> dict:
    return {"metric": metric, "status": "timeout", "value": None, "n_gpus": world, "reason": reason,
            "waited_s": round(waited_s, 1), "phases": phases}


class Heartbeat:
    """This rank's phase file + the watchdog (``start``)."""

    def __init__(self, rank: int, world: int, directory: Optional[str] = None, log_path: str = ""):
        self.rank, self.world = rank, world
        # optional per-rank phase history (one JSON line per phase; the rehearsal runs commit it)
        self.log_path = f"{log_path}.rank{rank}.jsonl" if log_path else ""
        self.dir = directory or default_dir()
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, f"rank{rank}")
        self.t0 = time.time()
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None
        self.phase("start")

    def phase(self, name: str) -> None:
        tmp = f"{self.path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump({"phase": name, "t": time.time(), "pid": os.getpid()}, f)
        os.replace(tmp, self.path)
        if self.log_path:
            with open(self.log_path, "a") as f:
                f.write(json.dumps({"rank": self.rank, "phase": name, "t": round(time.time(), 4)}) + "\n")

    def start(self, metric: str, stall_s: float, total_s: Optional[float] = None,
              on_timeout: Optional[Callable[[dict], None]] = None, poll_s: float = 1.0) -> None:
        """Watchdog: on a stall / deadline, report and ``os._exit(124)`` (a hung collective or
        kernel cannot be unwound; the process is ended without running further GPU work)."""
        def run():
            while not self._stop.wait(poll_s):
                now = time.time()
                prog = max(last_progress(self.dir, self.world), self.t0)
                reason = None
                if stall_s and now - prog > stall_s:
                    reason = f"no rank advanced for {now - prog:.0f} s (stall limit {stall_s:.0f} s)"
                elif total_s and now - self.t0 > total_s:
                    reason = f"job exceeded {total_s:.0f} s"
                if reason is None:
                    continue
                rec = timeout_record(metric, self.world, read_phases(self.dir, self.world), reason, now - self.t0)
                if on_timeout is not None:
                    try:
                        on_timeout(rec)
                    except Exception:  # noqa: BLE001 - reporting must not block the exit
                        pass
                if self.rank == 0:
                    sys.stdout.write(json.dumps(rec) + "\n")
                    sys.stdout.flush()
                sys.stderr.write(f"[rank {self.rank}] hang guard: {reason}; phases {json.dumps(rec['phases'])}\n")
                sys.stderr.flush()
                os._exit(124)
        self._th = threading.Thread(target=run, name="lp-hang-guard", daemon=True)
        self._th.start()

    def stop(self) -> None:
        self._stop.set()
