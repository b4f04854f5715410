#!/usr/bin/env python3
"""Cost of ONE BPG candidate walk on the GPU (bpg.hip), per program of the realistic library:
the cooperative walk (request path, N.bpg_cand_dev) and the one-lane walk (bulk path,
N.bpg_dedupe_dev) over one non-matching ASCII line of L bytes, L in --lens. Prints, per program,
the median kernel time (torch events around 20 launches, minus an empty launch) at each L and
the per-byte slope -- a request verifies only a handful of candidates, so one walk's latency IS
the kernel's time.

    python tools/bpg_probe.py --lens 32,128,512 --java-shape-rate 0.01
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="32,128,512")
    ap.add_argument("--java-shape-rate", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from log_parser_amd.models import bpg
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.native import N
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.utils.config import ScoringParams
    from log_parser_amd.utils.synth import realistic_library
    dev = torch.device("cuda", 0)
    sets, _ = realistic_library(1000, seed=7, java_shape_rate=args.java_shape_rate)
    lib = CompiledLibrary(sets, ScoringParams())
    dfa = lib.device_tables(dev)["dfa"]
    st = torch.cuda.current_stream().cuda_stream
    lens = [int(x) for x in args.lens.split(",")]

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        out = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            out.append(a.elapsed_time(b) * 1e3)
        return statistics.median(out)

    rows = []
    for L in lens:
        line = ("the quick brown fox jumps over a lazy dog 0123456789 " * (L // 50 + 1))[:L]
        data = (line + "\n").encode()
        t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        text = t.to(dev)
        ls = torch.zeros(1, dtype=torch.int64, device=dev)
        ll = torch.full((1,), L, dtype=torch.int32, device=dev)
        empty = torch.full((64,), -1, dtype=torch.int64, device=dev)
        base_c = timed(lambda: N.bpg_cand_dev(empty.data_ptr(), 64, text.data_ptr(), ls.data_ptr(), ll.data_ptr(),
                                              dfa, st))
        flag = torch.zeros(64, dtype=torch.uint8, device=dev)
        for r in lib.bpg_regs:
            c = torch.full((64,), -1, dtype=torch.int64, device=dev)

            def coop():
                c.fill_(-1)
                c[0] = (r << 32) | 0
                N.bpg_cand_dev(c.data_ptr(), 64, text.data_ptr(), ls.data_ptr(), ll.data_ptr(), dfa, st)
            t_coop = timed(coop) - base_c
            lbits = 1
            keys = torch.tensor([((r << lbits) | 0) << 1], dtype=torch.int64, device=dev)
            t_lane = timed(lambda: N.bpg_dedupe_dev(keys.data_ptr(), 1, lbits, text.data_ptr(), ls.data_ptr(),
                                                    ll.data_ptr(), dfa, flag.data_ptr(), st))
            info = bpg.program_info(lib.bpg_program(r))
            rows.append({"r": r, "L": L, "coop_us": round(t_coop, 2), "lane_us": round(t_lane, 2),
                         "pattern": lib.regexes[r].pattern[:50],
                         **{k: info[k] for k in ("words", "exceptions", "counters", "uniform", "unicode_word")}})
    for r in lib.bpg_regs:
        rr = [x for x in rows if x["r"] == r]
        slope = lambda key: (rr[-1][key] - rr[0][key]) / max(1, rr[-1]["L"] - rr[0]["L"])  # noqa: E731
        print(json.dumps({"r": r, "pattern": rr[0]["pattern"], "words": rr[0]["words"],
                          "exceptions": rr[0]["exceptions"], "counters": rr[0]["counters"],
                          "uniform": rr[0]["uniform"], "unicode_word": rr[0]["unicode_word"],
                          "coop_us": [x["coop_us"] for x in rr], "lane_us": [x["lane_us"] for x in rr],
                          "coop_ns_per_byte": round(1e3 * slope("coop_us"), 1),
                          "lane_ns_per_byte": round(1e3 * slope("lane_us"), 1)}), flush=True)


if __name__ == "__main__":
    main()
