"""Single-node rank launcher: one process per GPU, started by a parent that never touches the GPU.

``bench.py --gpus N`` (and any other entry point) can run without ``torch.distributed.run``: the
parent picks a free rendezvous port on 127.0.0.1, starts N fresh interpreters with the standard
``RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT`` environment and
exits with the first non-zero child status (the other ranks are terminated by their exact
process handles, never by pattern). The parent makes no HIP call: a process that has initialised
the GPU must not fork the ranks' interpreters, and each rank selects its own device
(``torch.cuda.set_device(LOCAL_RANK)``) and binds to its GPU's NUMA node.
"""
from __future__ import annotations

import contextlib
import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


HW_QUEUES = 8


def ensure_hw_queues(n: int = HW_QUEUES) -> int:
    """Give HIP at least ``n`` hardware queues per process (``GPU_MAX_HW_QUEUES``, HIP's default is 4).

    Must run before the process's first HIP call (it is read once, at runtime init). With 4 queues
    the streams of one rank -- compute, ingest copy, event D2H and RCCL's internal streams -- share
    queues, and the ingest copy then waits for the step's kernels instead of overlapping them: a
    world-1 RCCL group cost 23.5 -> 27.1 ms/step, and 8 queues remove it (profiles/r3_f). Child
    processes (ranks, the server) inherit the setting. Returns the value in effect.
    """
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        cur = 0
    if n <= 0:
        return cur
    if cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)
        cur = n
    return cur


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def under_launcher() -> bool:
    """True when this process already is one rank of a launched job."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def rank_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def spawn_local_ranks(argv: Sequence[str], world: int, poll_s: float = 0.2,
                      timeout_s: Optional[float] = None) -> int:
    """Run ``python argv...`` as ``world`` ranks on this node; returns the job's exit status."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    try:
        for r in range(world):
            # rank 0 keeps the parent's stdout (the one JSON line); other ranks' stdout -> stderr
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, world, port),
                                          stdout=None if r == 0 else sys.stderr))
        t0 = time.monotonic()
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                return 124
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


@contextlib.contextmanager
def stdout_to_stderr():
    """Point file descriptor 1 at stderr for the duration (native libraries such as RCCL print
    banners with printf; a bench's stdout must carry only its JSON line)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
