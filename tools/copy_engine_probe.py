"""Which engine moves a host -> device copy: SDMA (a memory-copy record) or a blit kernel
(``__amd_rocclr_copyBuffer`` on the CUs)? One copy per case, each of a distinct size, separated by
a sync and a pause, so the trace's records map back to the cases by size and order.
Run under ``rocprofv3 --kernel-trace --memory-copy-trace`` (tools/gpu_copy_probe.sh); prints one
JSON line per case (host-timed GB/s)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from log_parser_amd.native import N  # noqa: E402
from log_parser_amd.utils.hostmem import registered_empty  # noqa: E402

MB = 1 << 20


def backlog():
    """Copies queued behind each other (the bench's prefetch: the next step's H2D is queued while the
    current one still runs): which of them become blit kernels?"""
    dev = torch.empty(2800 * MB, dtype=torch.uint8, device="cuda")
    host = registered_empty(1400 * MB)
    host.fill_(7)
    side, comp = torch.cuda.Stream(), torch.cuda.Stream()
    groups = [("2x1333", [1333] * 2), ("3x1333", [1333] * 3), ("8x256", [256] * 8), ("12x64", [64] * 12)]
    case = 100
    for name, sizes in groups:
        torch.cuda.synchronize()
        time.sleep(0.05)
        t0 = time.perf_counter()
        tot = 0
        with torch.cuda.stream(side):
            for k, mb in enumerate(sizes):
                case += 1
                n = mb * MB + case * 4096
                o = (k % 2) * 1400 * MB
                dev[o:o + n].copy_(host[:n], non_blocking=True)
                tot += n
        side.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"group": name, "last_case": case, "bytes": tot, "GBps": round(tot / dt / 1e9, 2)}), flush=True)
    # dependencies as in the bench: each copy waits for a compute-stream event, compute waits for it
    torch.cuda.synchronize()
    time.sleep(0.05)
    ev_free = [torch.cuda.Event(), torch.cuda.Event()]
    x = torch.empty(64 * MB, device="cuda")
    for k in range(6):
        case += 1
        n = 1333 * MB + case * 4096
        o = (k % 2) * 1400 * MB
        with torch.cuda.stream(side):
            if k >= 2:
                side.wait_event(ev_free[k % 2])
            dev[o:o + n].copy_(host[:n], non_blocking=True)
            ready = torch.cuda.Event()
            ready.record(side)
        comp.wait_event(ready)
        with torch.cuda.stream(comp):
            for _ in range(20):
                x.mul_(1.0001)
            ev_free[k % 2].record(comp)
    torch.cuda.synchronize()
    print(json.dumps({"group": "dep6x1333", "last_case": case}), flush=True)


def main():
    if "--backlog" in sys.argv:
        return backlog()
    dev = torch.empty(1400 * MB, dtype=torch.uint8, device="cuda")
    side = torch.cuda.Stream()
    big = 1333 * MB
    kinds = {"hostmalloc": torch.empty(big + 7 * MB, dtype=torch.uint8, pin_memory=True),
             "registered": registered_empty(big + 7 * MB)}
    for t in kinds.values():
        t.fill_(7)
    case = 0
    for kind, host in kinds.items():
        for size_mb in (1333, 256, 64, 4):
            for api in ("torch", "native"):
                for where in ("side", "default"):
                    case += 1
                    n = size_mb * MB + case * 4096          # distinct size per case
                    st = side if where == "side" else torch.cuda.current_stream()
                    torch.cuda.synchronize()
                    time.sleep(0.02)
                    t0 = time.perf_counter()
                    with torch.cuda.stream(st):
                        if api == "torch":
                            dev[:n].copy_(host[:n], non_blocking=True)
                        else:
                            N.copy_h2d(dev.data_ptr(), host.data_ptr(), n, st.cuda_stream)
                    st.synchronize()
                    dt = time.perf_counter() - t0
                    print(json.dumps({"case": case, "kind": kind, "api": api, "stream": where, "bytes": n,
                                      "GBps": round(n / dt / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
