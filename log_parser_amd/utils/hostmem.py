"""Page-locked host buffers for bulk host-to-device copies.

Two kinds of pinned memory behave differently on the copy path (ROCm 7, MI355X):
* ``torch.empty(..., pin_memory=True)`` (hipHostMalloc) -- ROCclr moves it with a BLIT KERNEL
  (``__amd_rocclr_copyBuffer``): a 1.33 GB H2D ran 23 ms as a kernel occupying CUs next to the
  step's own kernels, which then ran slower (k_prefilter 1.03 vs 0.67 ms, profiles/r4_c);
* ordinary pages registered with ``hipHostRegister`` -- moved by the SDMA engines, no CU time,
  at the same ~57 GB/s (profiles/r4_b).
``registered_empty`` gives the second kind (an anonymous mapping, registered in place, unregistered
and unmapped when the tensor's owner goes away), or falls back to the first when registration is
refused or no GPU is present.
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
