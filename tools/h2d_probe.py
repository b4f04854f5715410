"""Host->device ingest bandwidth probe: SDMA copy (1 / 2 / 4 streams). (The k_pull kernel -- the GPU
reading pinned host memory -- measured 55.6 GB/s vs 57.6 SDMA in round 1 and was removed.)
(GPU reads pinned host memory over PCIe), with and without NUMA binding. Prints JSON lines."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from log_parser_amd.native import N  # noqa: E402
from log_parser_amd.utils.numa import bind_to_gpu_numa, gpu_numa_cpus  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    bind = "--bind" in sys.argv
    cpus = bind_to_gpu_numa(0) if bind else None
    print(json.dumps({"bind": bind, "gpu_local_cpus": len(gpu_numa_cpus(0)), "bound_to": len(cpus) if cpus else None}),
          flush=True)
    n = 1_333_838_336
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.random_(0, 255)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    res = {}
    res["sdma_1"] = timeit(lambda: dev.copy_(host, non_blocking=True))
    for k in (2, 4):
        streams = [torch.cuda.Stream() for _ in range(k)]
        step = n // k

        def multi():
            cur = torch.cuda.current_stream()
            for j, s in enumerate(streams):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    dev[j * step:(j + 1) * step].copy_(host[j * step:(j + 1) * step], non_blocking=True)
            for s in streams:
                cur.wait_stream(s)
        res[f"sdma_{k}"] = timeit(multi)
    assert torch.equal(dev[:1 << 20].cpu(), host[:1 << 20])
    assert torch.equal(dev[-(1 << 20):].cpu(), host[-(1 << 20):])
    print(json.dumps({k: {"ms": round(v * 1e3, 3), "GBps": round(n / v / 1e9, 2)} for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
