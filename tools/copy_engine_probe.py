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


def main():
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
