"""A/B of the whole-text engines for literal-free regexes: multi-regex DFA scan groups
(csrc/kernels/scan_multi.hip), the MFMA NFA state-transition kernel (csrc/kernels/nfa_mfma.hip)
and bit-parallel Glushkov programs (csrc/kernels/bpg.h, one lane per line) on N literal-free
regexes over every line of a synthetic log.

    python tools/scan_ab.py --regexes 64 --lines 2500000 [--engine dfa|mfma|bpg|both|all] [--reps 10]

Prints one JSON line: per-engine kernel time (median of --reps, HIP events), hits (both engines
must agree), groups. Used for the crossover table in docs/PERFORMANCE.md and under rocprofv3 PMC.
"""
import argparse
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.models.nfa import build_group, fits_group, pack_groups  # noqa: E402
from log_parser_amd.models.schema import PatternSet  # noqa: E402
from log_parser_amd.native import N  # noqa: E402
from log_parser_amd.ops import kernels as K  # noqa: E402
from log_parser_amd.utils.config import ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import _literal_free, make_log  # noqa: E402


def library(n):
    rng = random.Random(5)
    pats, trig, seen = [], [], set()
    i = 0
    while len(pats) < n:
        rx, sample = _literal_free(rng, i)
        i += 1
        if rx in seen:
            continue
        seen.add(rx)
        pats.append({"id": f"lf-{len(pats)}", "name": rx, "severity": "HIGH",
                     "primary_pattern": {"regex": rx, "confidence": 0.5}})
        trig.append({"sample": sample, "secondary": [], "sequence": []})
    ps = PatternSet.model_validate({"metadata": {"library_id": "lf"}, "patterns": pats})
    return [ps], trig


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts)), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regexes", type=int, default=64)
    ap.add_argument("--lines", type=int, default=2_500_000)
    ap.add_argument("--engine", default="both", choices=["dfa", "mfma", "bpg", "both", "all"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--group-regs", type=int, default=0, help="members per scan group (0: the library default)")
    args = ap.parse_args()
    if args.group_regs:
        CompiledLibrary.SCAN_GROUP_REGS = args.group_regs
    dev = torch.device("cuda", 0)
    sets, trig = library(args.regexes)
    lib = CompiledLibrary(sets, ScoringParams())
    block = make_log(min(args.lines, 250_000), trig, seed=3, hit_rate=0.01).encode()
    reps = max(1, args.lines // block.count(b"\n"))
    data = block * reps
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(dev)
    ls, ll = K.split_lines(t, len(data))
    L = ls.numel()
    rec = {"regexes": args.regexes, "lines": L, "bytes": len(data), "group_regs": CompiledLibrary.SCAN_GROUP_REGS}
    tabs = lib.device_tables(dev)
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    hits = {}
    if args.engine in ("dfa", "both", "all"):
        def run_dfa():
            outs = []
            for sp in tabs["scan_passes"]:
                per_cu = max(1, min(2, (160 << 10) // (sp[1] * 4)))
                outs.append(K.scan_multi(t, len(data), ls, ll, sp, max(1024, L >> 4), n_cus * per_cu))
            return torch.cat(outs) if outs else torch.empty(0, dtype=torch.int64, device=dev)
        us, h = timed(run_dfa, args.reps)
        hits["dfa"] = torch.sort(h).values.cpu()
        rec["dfa_us"] = round(us, 1)
        rec["dfa_groups"] = len(lib.scan_groups)
        rec["dfa_passes"] = len(lib.scan_passes)
        rec["dfa_states"] = [d["nstates"] for _, d in lib.scan_groups]
        rec["dfa_single"] = len(lib.scan_regs_single)
    if args.engine in ("mfma", "both", "all"):
        members = []
        for r in lib.scan_regs:
            d = N.compile_regex(lib.regexes[r].pattern, 4, 4096)
            if fits_group(d):
                members.append((r, d))
        groups = pack_groups(members)
        tabs_np, ncls = zip(*[build_group(g) for g in groups])
        gt = torch.from_numpy(np.concatenate(tabs_np).view(np.int64)).to(dev)
        per_cls = {}
        for gi, k in enumerate(ncls):
            per_cls.setdefault(k, []).append(gi)
        lists = {k: torch.tensor(v, dtype=torch.int32, device=dev) for k, v in per_cls.items()}

        def run_mfma():
            return torch.cat([K.nfa_scan(gt, gl, k, t, ls, ll, max(1024, L >> 4)) for k, gl in lists.items()])
        us, h = timed(run_mfma, args.reps)
        hits["mfma"] = torch.sort(h).values.cpu()
        rec["mfma_us"] = round(us, 1)
        rec["mfma_groups"] = len(groups)
        rec["mfma_regexes"] = len(members)
    if args.engine in ("bpg", "all"):
        blib = CompiledLibrary(sets, ScoringParams(), max_dfa_states=4)      # every regex -> BPG program
        btabs = blib.device_tables(dev)
        regs = torch.tensor(blib.bpg_regs, dtype=torch.int32, device=dev)

        def run_bpg():
            return K.scan(t, ls, ll, regs, btabs["dfa"], max(1024, L >> 4))
        us, h = timed(run_bpg, args.reps)
        hits["bpg"] = torch.sort(h).values.cpu()
        rec["bpg_us"] = round(us, 1)
        rec["bpg_regexes"] = len(blib.bpg_regs)
    for k, v in hits.items():
        rec[f"{k}_hits"] = int(v.numel())
    if len(hits) >= 2 and "dfa" in hits:
        rec["agree"] = {k: bool(torch.equal(hits["dfa"], v)) for k, v in hits.items() if k != "dfa"
                        and (k != "mfma" or rec.get("mfma_regexes") == len(lib.scan_regs))}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
