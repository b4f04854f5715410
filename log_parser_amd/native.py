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


def load():
    global _mod
    if _mod is not None:
        return _mod
    if os.environ.get("LP_NO_AUTOBUILD", "0") != "1" and _needs_build():
        from . import _build
        _build.build()
    _mod = importlib.import_module("log_parser_amd._lpnative")
    # CPU-backend worker threads: this process's CPU share, at most 16 (LP_HOST_THREADS overrides)
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 8)
    _mod.set_host_threads(int(os.environ.get("LP_HOST_THREADS", min(16, n))))
    return _mod


class _Lazy:
    def __getattr__(self, name):
        return getattr(load(), name)


N = _Lazy()
