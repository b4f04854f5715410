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
                      timeout_s: Optional[float] = None, stall_s: Optional[float] = None,
                      metric: str = "") -> int:
    """Run ``python argv...`` as ``world`` ranks on this node; returns the job's exit status.

    Hang guard (backstop of the ranks' own watchdogs, ``utils/heartbeat.py``): the ranks write
    their phases into a fresh heartbeat directory; past ``timeout_s`` in total, or ``stall_s``
    without any rank advancing, the parent prints one ``{"status": "timeout", "phases": ...}``
    JSON line, ends the ranks by their exact handles and returns 124."""
    import shutil
    import tempfile
    from .heartbeat import ENV_DIR, last_progress, read_phases, timeout_record
    port = free_port()
    hb_dir = tempfile.mkdtemp(prefix="lp-heartbeat-")
    procs: List[subprocess.Popen] = []
    try:
        for r in range(world):
            env = rank_env(r, world, port)
            env[ENV_DIR] = hb_dir
            # rank 0 keeps the parent's stdout (the one JSON line); other ranks' stdout -> stderr
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=env,
                                          stdout=None if r == 0 else sys.stderr))
        t0 = time.monotonic()
        w0 = time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            reason = None
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                reason = f"job exceeded {timeout_s:.0f} s"
            elif stall_s is not None and time.time() - max(last_progress(hb_dir, world), w0) > stall_s:
                reason = f"no rank advanced for {stall_s:.0f} s"
            if reason is not None:
                import json
                rec = timeout_record(metric, world, read_phases(hb_dir, world), reason + " (launcher)",
                                     time.monotonic() - t0)
                sys.stdout.write(json.dumps(rec) + "\n")
                sys.stdout.flush()
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
        shutil.rmtree(hb_dir, ignore_errors=True)


def inject_fault(rank: int, step: int) -> None:
    """Fault injection for the multi-process tests: ``LP_FAULT_RANK=k LP_FAULT_STEP=n`` makes rank
    ``k`` exit (status 17) at the start of step ``n``; ``LP_FAULT_MODE=hang`` makes it stop
    responding for ``LP_FAULT_HANG_S`` seconds instead (then exit 18)."""
    r, s = os.environ.get("LP_FAULT_RANK"), os.environ.get("LP_FAULT_STEP")
    if r is None or s is None or int(r) != rank or int(s) != step:
        return
    if os.environ.get("LP_FAULT_MODE", "exit") == "hang":
        time.sleep(float(os.environ.get("LP_FAULT_HANG_S", "86400")))
        os._exit(18)
    os._exit(17)


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
