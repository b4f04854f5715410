"""What the threads of a process are doing, sampled from /proc (config-5 serving diagnostics).

``ThreadSampler(pids).start()`` reads, every ``period_s``, each thread's name
(``/proc/<pid>/task/<tid>/comm``), scheduler state (``stat``), kernel wait channel (``wchan``) and
current system call (``syscall``, first field), and ``summary()`` counts the samples per thread
name and (state, wait) -- e.g. ``lp-io3: S ep_poll 812`` -- so a slow burst shows which wait its
serving threads sit in: the accept backlog, epoll wake-ups, the pump's condition variable (futex),
the GIL (futex), or running (R). ``set_os_thread_name`` names the calling OS thread (15 bytes),
so Python threads show up by role instead of as "python".
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from collections import Counter, defaultdict
from typing import Dict, List

_SYSCALLS = {0: "read", 1: "write", 7: "poll", 23: "select", 35: "nanosleep", 202: "futex", 232: "epoll_wait",
             281: "epoll_pwait", 288: "accept4", 43: "accept", 44: "sendto", 45: "recvfrom", 46: "sendmsg",
             47: "recvmsg", 16: "ioctl", 230: "clock_nanosleep", 228: "clock_gettime", 24: "sched_yield",
             441: "epoll_pwait2"}


def set_os_thread_name(name: str) -> None:
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(15, ctypes.c_char_p(name.encode()[:15]), 0, 0, 0)      # PR_SET_NAME
    except (OSError, AttributeError):
        pass


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


class ThreadSampler:
    def __init__(self, pids: List[int], period_s: float = 0.001):
        self.pids = list(pids)
        self.period_s = period_s
        self.counts: Dict[str, Counter] = defaultdict(Counter)
        self.samples = 0
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, name="lp-sampler", daemon=True)

    def start(self) -> "ThreadSampler":
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._th.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.is_set():
            for pid in self.pids:
                try:
                    tids = os.listdir(f"/proc/{pid}/task")
                except OSError:
                    continue
                for tid in tids:
                    base = f"/proc/{pid}/task/{tid}"
                    comm = _read(base + "/comm") or "?"
                    st = _read(base + "/stat")
                    state = st[st.rfind(")") + 2] if ")" in st else "?"
                    if state == "R":
                        what = "running"
                    else:
                        wchan = _read(base + "/wchan") or "0"
                        sc = _read(base + "/syscall").split(" ")[0]
                        name = _SYSCALLS.get(int(sc), sc) if sc.lstrip("-").isdigit() else sc
                        what = f"{name}/{wchan}" if wchan not in ("0", "") else name
                    self.counts[f"{pid}:{comm}"][f"{state} {what}"] += 1
            self.samples += 1
            time.sleep(self.period_s)

    def summary(self, top: int = 4) -> Dict[str, dict]:
        """{pid:thread-name: {"samples": n, "top": [[state wait, share], ...]}}, threads of one name
        merged (e.g. the IO threads), busiest first."""
        by_name: Dict[str, Counter] = defaultdict(Counter)
        for k, c in self.counts.items():
            by_name[k.split(":", 1)[0] + ":" + k.split(":", 1)[1].rstrip("0123456789")] += c
        out = {}
        for k, c in sorted(by_name.items(), key=lambda kv: -sum(kv[1].values())):
            n = sum(c.values())
            out[k] = {"samples": n, "top": [[w, round(m / n, 3)] for w, m in c.most_common(top)]}
        return out
