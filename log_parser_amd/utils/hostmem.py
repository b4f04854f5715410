"""Page-locked host buffers for bulk host-to-device copies.

``registered_empty`` gives ordinary pages registered in place with ``hipHostRegister`` (an
anonymous mapping, unregistered and unmapped when the tensor's owner goes away), or falls back to
torch's pinned allocator (hipHostMalloc) when registration is refused or no GPU is present. Both
kinds are copied by the SDMA engines at ~57 GB/s (profiles/r4_c: copy-engine probes over both kinds,
torch and native copies, queued copies; the HIP runtime's own log of the bench). A blit kernel
(``__amd_rocclr_copyBuffer``) replaces the SDMA copy only when the HSA copy call fails, which was
seen only under the profiler. Registration lets a buffer be sized and laid out by the caller (an
mmap of any size, a page-locked view of memory that already exists).
"""
from __future__ import annotations

import mmap
import weakref

import numpy as np
import torch


class _Registered:
    def __init__(self, nbytes: int):
        from ..native import N
        self.map = mmap.mmap(-1, max(int(nbytes), 1))
        self.arr = np.frombuffer(self.map, dtype=np.uint8)[:nbytes]
        self.ok = bool(N.host_register(self.arr.ctypes.data, max(int(nbytes), 1)))
        if self.ok:
            # unregister before the mapping goes (the finalizer holds the mapping until then)
            weakref.finalize(self, lambda m, p: N.host_unregister(p), self.map, self.arr.ctypes.data)


def registered_empty(nbytes: int) -> torch.Tensor:
    """A uint8 CPU tensor of ``nbytes`` in registered (SDMA-copied) page-locked memory; the tensor
    keeps the registration alive. Falls back to torch's pinned allocator."""
    if torch.cuda.is_available() and nbytes > 0:
        r = _Registered(nbytes)
        if r.ok:
            t = torch.from_numpy(r.arr)
            t._lp_registration = r          # lifetime: the registration lives as long as the tensor
            return t
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
