"""Loader for the in-tree native extension (``_lpnative.so``).

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and the
extension links the same SONAME, so the dynamic loader reuses torch's HIP runtime instead of
loading a second one (one runtime => shared streams, allocator and device context).
If the extension is missing or older than its sources it is (re)built with hipcc.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension import, see module docstring)

_mod = None


def _needs_build() -> bool:
    from . import _build
    if not os.path.exists(_build.OUT):
        return True
    t = os.path.getmtime(_build.OUT)
    for rel, _ in _build.SOURCES:
        p = os.path.join(_build.CSRC, rel)
        if os.path.exists(p) and os.path.getmtime(p) > t:
            return True
    return any(os.path.getmtime(h) > t for h in _build._headers())


def host_thread_budget() -> int:
    """Worker threads for native host loops (packing, JSON emission, CPU twins): this process's
    share of the CPU budget (cgroup quota aware; one of LP_SERVE_NPROC serving processes gets
    1/n of it), at most 16."""
    from .utils.numa import cpu_budget
    nproc = max(1, int(os.environ.get("LP_SERVE_NPROC", "1") or 1))
    return max(1, min(16, cpu_budget() // nproc))


def load():
    global _mod
    if _mod is not None:
        return _mod
    if os.environ.get("LP_NO_AUTOBUILD", "0") != "1" and _needs_build():
        from . import _build
        _build.build()
    _mod = importlib.import_module("log_parser_amd._lpnative")
    # CPU-backend worker threads: this process's CPU share, at most 16 (LP_HOST_THREADS overrides)
    _mod.set_host_threads(int(os.environ.get("LP_HOST_THREADS", host_thread_budget())))
    return _mod


class _Lazy:
    def __getattr__(self, name):
        return getattr(load(), name)


N = _Lazy()
