"""Host staging probe for the streaming path: pinned allocation, host->pinned copy throughput
(torch copy_, numpy with N threads), hipHostRegister rate, H2D from registered memory."""
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, ".")


def t(fn, reps=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main():
    n = 512 << 20
    src = np.random.randint(0, 255, size=n, dtype=np.uint8)
    srct = torch.from_numpy(src)
    out = {"torch_threads": torch.get_num_threads()}
    t0 = time.perf_counter()
    pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    out["pin_alloc_512MB_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    p2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    out["pin_alloc2_512MB_ms"] = (time.perf_counter() - t0) * 1e3
    del p2
    out["torch_copy_GBps"] = n / t(lambda: pinned.copy_(srct)) / 1e9
    pn = pinned.numpy()
    for th in (4, 8, 16):
        ex = ThreadPoolExecutor(th)
        step = n // th

        def par():
            list(ex.map(lambda j: np.copyto(pn[j * step:(j + 1) * step], src[j * step:(j + 1) * step]), range(th)))
        out[f"np_copy_{th}thr_GBps"] = n / t(par) / 1e9
        ex.shutdown()
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    big = np.random.randint(0, 255, size=2 << 30, dtype=np.uint8)
    cr = torch.cuda.cudart()
    t0 = time.perf_counter()
    rc = cr.cudaHostRegister(big.ctypes.data, big.nbytes, 0)
    out["register_2GB_ms"] = (time.perf_counter() - t0) * 1e3
    out["register_rc"] = int(rc) if not isinstance(rc, tuple) else [int(x) for x in rc]
    bt = torch.from_numpy(big)

    def h2d():
        dev.copy_(bt[:n], non_blocking=True)
        torch.cuda.synchronize()
    out["h2d_registered_GBps"] = n / t(h2d) / 1e9
    out["h2d_pinned_GBps"] = n / t(lambda: (dev.copy_(pinned, non_blocking=True), torch.cuda.synchronize())) / 1e9
    t0 = time.perf_counter()
    cr.cudaHostUnregister(big.ctypes.data)
    out["unregister_2GB_ms"] = (time.perf_counter() - t0) * 1e3
    out["h2d_pageable_GBps"] = n / t(h2d) / 1e9
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
