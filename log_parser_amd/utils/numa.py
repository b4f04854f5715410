"""Pin a rank's host threads (and therefore its pinned staging buffers) to its GPU's NUMA node.

Ingest is PCIe-bound (docs/PERFORMANCE.md): every log byte crosses the host->GPU link once.
Pinned buffers are placed on the NUMA node of the allocating thread, so a rank whose staging
memory sits on the far socket pays an extra inter-socket hop on every H2D transfer -- and with 8
ranks, half of them would. Call :func:`bind_to_gpu_numa` before allocating pinned memory.
"""
from __future__ import annotations

import os
from typing import Optional, Set


def _parse_cpulist(s: str) -> Set[int]:
    out: Set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def gpu_pci_path(index: int) -> Optional[str]:
    import torch
    try:
        p = torch.cuda.get_device_properties(index)
        dom, bus, dev = int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)
    except Exception:  # noqa: BLE001 - older torch / no device
        return None
    path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.0"
    return path if os.path.isdir(path) else None


def gpu_numa_cpus(index: int) -> Set[int]:
    path = gpu_pci_path(index)
    if path is None:
        return set()
    try:
        with open(os.path.join(path, "local_cpulist")) as f:
            return _parse_cpulist(f.read())
    except OSError:
        return set()


def gpu_numa_node(index: int) -> int:
    """NUMA node of GPU ``index`` (-1 when unknown)."""
    path = gpu_pci_path(index)
    if path is None:
        return -1
    try:
        with open(os.path.join(path, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def bind_to_gpu_numa(index: int) -> Optional[Set[int]]:
    """Restrict this process to the CPUs local to GPU ``index`` (intersected with the CPUs it may
    already use). Returns the new CPU set, or None when nothing was changed."""
    if os.environ.get("LP_NUMA_BIND", "1") == "0":
        return None
    local = gpu_numa_cpus(index)
    try:
        allowed = os.sched_getaffinity(0)
    except AttributeError:
        return None
    cpus = local & allowed
    if not cpus or cpus == allowed:
        return None
    os.sched_setaffinity(0, cpus)
    return cpus


def l3_groups(cpus: Set[int]) -> list:
    """``cpus`` grouped by shared last-level cache (an EPYC CCD's L3: the cores that exchange a
    request's bytes cheaply), largest group first; one group when the topology is not visible."""
    groups = {}
    for c in sorted(cpus):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                key = frozenset(_parse_cpulist(f.read().strip()))
        except OSError:
            key = frozenset()
        groups.setdefault(key, set()).add(c)
    return sorted(groups.values(), key=lambda g: (-len(g), min(g)))


def one_per_core(cpus: Set[int]) -> Set[int]:
    """``cpus`` with one hardware thread per physical core (the lowest sibling present): threads that
    work at the same time -- the HTTP IO thread receiving a body and the pump decoding it -- on SMT
    siblings of one core share its execution units (the receive ran ~2x slower, profiles/r6_e)."""
    out: Set[int] = set()
    seen = set()
    for c in sorted(cpus):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                sib = frozenset(_parse_cpulist(f.read().strip()))
        except OSError:
            sib = frozenset([c])
        if sib in seen:
            continue
        seen.add(sib)
        out.add(c)
    return out


def cpu_limits() -> dict:
    """The two limits behind ``cpu_budget``: the affinity set and the cgroup CPU quota (None: none)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"affinity": aff, "quota_cpus": _cgroup_quota()}


def _cgroup_quota() -> Optional[float]:
    """The cgroup CPU quota in CPUs (v2 ``cpu.max``, v1 ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``),
    None when unlimited or not visible."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return q / p if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None


def cgroup_throttling() -> dict:
    """CFS bandwidth throttling of this cgroup so far (cgroup v2 ``cpu.stat``, v1 ``cpu/cpu.stat``):
    periods in which the group ran out of quota and the time its threads were held off -- a burst
    that runs more threads than the quota stalls every thread for the rest of each period."""
    for path, scale in (("/sys/fs/cgroup/cpu.stat", 1e-3), ("/sys/fs/cgroup/cpu/cpu.stat", 1e-6)):
        try:
            with open(path) as f:
                kv = dict(line.split()[:2] for line in f if line.strip())
        except (OSError, ValueError):
            continue
        t = kv.get("throttled_usec", kv.get("throttled_time"))
        return {"periods": int(kv.get("nr_periods", 0)), "throttled_periods": int(kv.get("nr_throttled", 0)),
                "throttled_ms": float(t) * scale if t is not None else 0.0}
    return {}


def cpu_budget() -> int:
    """CPUs this process can actually use: its affinity set, capped by a cgroup CPU quota
    (``cpu.max``, v2, or ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``, v1) -- a container's
    ``os.cpu_count()`` shows the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_quota()
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)
