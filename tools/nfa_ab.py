"""Per-shape A/B of the two automaton engines for regexes whose DFA blows up: bit-parallel Glushkov
programs (BPG, csrc/kernels/bpg.hip) against the NFA state-transition GEMM on the matrix cores
(MFMA, csrc/kernels/nfa_mfma.hip), on the shapes small enough for the MFMA kernel's 64-position
groups (the production route sends larger ones to BPG only).

Two modes per shape, same regexes, same text, hits compared exactly:
  * scan   -- every line (literal-free regexes): k_bpg_scan (one lane per line) vs k_nfa_mfma over
              all lines (16 lines per wave per MFMA tile);
  * verify -- prefilter-candidate lines only (the production route of regexes with a literal):
              the cooperative walk (bpg_cand_dev, a lane group per line) vs k_nfa_mfma over a line
              list, for every (regex, candidate line) pair.

    python tools/nfa_ab.py [--lines 1000000] [--cands 20000] [--reps 5] [--engine both|bpg|mfma]

Prints one JSON line per shape (kernel us = median of --reps, HIP events). Run under rocprofv3
--pmc with --engine mfma / bpg for the matrix-core and VALU counters (profiles/r3_o)."""
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

TOKS = ["alpha", "bravo", "cargo", "delta", "ember", "fjord", "gamma", "hotel"]
# shape name -> template with {t} = a per-regex token (8 regexes per shape)
SHAPES = {
    "bounded_gap": r"{t} refused.{{0,12}}port",
    "two_gaps": r"err.{{0,6}}{t}.{{0,6}}retry",
    "repeated_group": r"(\w+\.){{2,}}{t}Ex",
    "ip_boundary": r"\b\d{{1,3}}(?:\.\d{{1,3}}){{3}}\b.{{0,4}}{t}",
    "alternation_loop": r"(?:ab|{t})+d.{{0,8}}e",
    # the round-3 review's shapes, as written and scaled to the MFMA kernel's 64
    # positions: the unscaled ones and the code-point ones are recorded as not runnable on MFMA
    "r3_refused_600": r"Connection {t} refused.{{0,600}}port \d+",
    "r3_gap_pair_300": r"error.{{0,300}}{t}.{{0,300}}retry",
    "r3_refused_scaled": r"{t} refused.{{0,40}}port \d+",
    "r3_gap_pair_scaled": r"error.{{0,20}}{t}.{{0,20}}retry",
    "r3_unicode_letters": r"\p{{L}}+{t}Exception",
    "r3_multiline": r"(?m)^{t}ERROR$",
    "r3_java_dot": r"a.{{0,8}}{t}b",
}
FILL = ("the quick brown fox jumps over the lazy dog 10.0.0.7 port 8443 at com.acme.Foo. "
        "error while calling upstream, will retry in 5s refused by peer abd e")


def make_text(rng, n_lines, toks):
    words = FILL.split(" ") + toks + [t + "Ex" for t in toks] + ["refused", "retry", "err", "port"]
    out = []
    for _ in range(n_lines):
        out.append(" ".join(rng.choice(words) for _ in range(rng.randint(3, 18))))
    return "\n".join(out).encode()


def timed(fn, reps):
    ts = []
    out = None
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
    ap.add_argument("--lines", type=int, default=1_000_000)
    ap.add_argument("--cands", type=int, default=20_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--engine", default="both", choices=["both", "bpg", "mfma"])
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--library", default="", choices=["", "realistic"],
                    help="instead of --shapes: the bench library's own BPG programs (realistic_library(1000, "
                         "seed=7), bench.py's), one record per program: MFMA-runnable or why not, and for "
                         "the runnable ones the same scan / verify A/B on the bench's own text")
    args = ap.parse_args()
    if args.library:
        return library_ab(args)
    dev = torch.device("cuda", 0)
    rng = random.Random(7)
    blob = make_text(rng, min(args.lines, 200_000), TOKS)
    reps = max(1, args.lines // (blob.count(b"\n") + 1))
    data = b"\n".join([blob] * reps)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(dev)
    ls, ll = K.split_lines(t, len(data))
    L = ls.numel()
    stream = torch.cuda.current_stream().cuda_stream
    for shape in args.shapes.split(","):
        pats = [SHAPES[shape].format(t=tok) for tok in TOKS]
        ps = PatternSet.model_validate({"metadata": {"library_id": shape}, "patterns": [
            {"id": f"{shape}-{i}", "name": p, "severity": "HIGH", "primary_pattern": {"regex": p, "confidence": 0.5}}
            for i, p in enumerate(pats)]})
        lib = CompiledLibrary([ps], ScoringParams(), max_dfa_states=4)     # every regex -> a BPG program
        rec = {"shape": shape, "regex": pats[0], "lines": L, "bytes": len(data)}
        members = []
        for r in lib.bpg_regs:
            d = N.compile_regex(lib.regexes[r].pattern, 4, 4096)
            if fits_group(d):
                members.append((r, d))
        rec["bpg_regexes"] = len(lib.bpg_regs)
        rec["mfma_regexes"] = len(members)
        rec["positions"] = [int(d["npos"]) for _, d in members]
        if len(members) != len(lib.bpg_regs):
            rec["skipped"] = "some regexes exceed the MFMA kernel's 64 positions"
            print(json.dumps(rec), flush=True)
            continue
        groups = pack_groups(members)
        tabs_np, ncls = zip(*[build_group(g) for g in groups])
        gt = torch.from_numpy(np.concatenate(tabs_np).view(np.int64)).to(dev)
        per_cls = {}
        for gi, k in enumerate(ncls):
            per_cls.setdefault(k, []).append(gi)
        lists = {k: torch.tensor(v, dtype=torch.int32, device=dev) for k, v in per_cls.items()}
        rec["mfma_groups"] = len(groups)
        btabs = lib.device_tables(dev)
        regs = torch.tensor(lib.bpg_regs, dtype=torch.int32, device=dev)
        cap = max(4096, L * len(pats) // 4)
        hits = {}
        # ---- scan: every line
        if args.engine in ("both", "bpg"):
            us, h = timed(lambda: K.scan(t, ls, ll, regs, btabs["dfa"], cap), args.reps)
            rec["scan_bpg_us"] = round(us, 1)
            hits["bpg"] = torch.sort(h).values.cpu()
        if args.engine in ("both", "mfma"):
            us, h = timed(lambda: torch.cat([K.nfa_scan(gt, gl, k, t, ls, ll, cap) for k, gl in lists.items()]),
                          args.reps)
            rec["scan_mfma_us"] = round(us, 1)
            hits["mfma"] = torch.sort(h).values.cpu()
        for k, v in hits.items():
            rec[f"scan_{k}_hits"] = int(v.numel())
        if len(hits) == 2:
            rec["scan_agree"] = bool(torch.equal(hits["bpg"], hits["mfma"]))
        # ---- verify: candidate lines (every regex x the same random line sample)
        C = min(args.cands, L)
        lines = torch.tensor(sorted(rng.sample(range(L), C)), dtype=torch.int32, device=dev)
        pairs = (regs.to(torch.int64)[:, None] << 32 | lines.to(torch.int64)[None, :]).reshape(-1)
        vh = {}
        if args.engine in ("both", "bpg"):
            def run_bpg():
                c = pairs.clone()
                N.bpg_cand_dev(c.data_ptr(), c.numel(), t.data_ptr(), ls.data_ptr(), ll.data_ptr(), btabs["dfa"], stream)
                return c[c >= 0]
            us, h = timed(run_bpg, args.reps)
            rec["verify_bpg_us"] = round(us, 1)
            vh["bpg"] = torch.sort(h).values.cpu()
        if args.engine in ("both", "mfma"):
            def run_mfma():
                outs = []
                for k, gl in lists.items():
                    out = torch.empty(C * len(pats) + 1, dtype=torch.int64, device=dev)
                    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
                    N.nfa(gt.data_ptr(), gl.data_ptr(), gl.numel(), k, lines.data_ptr(), C, t.data_ptr(), ls.data_ptr(),
                          ll.data_ptr(), 0, out.data_ptr(), out.numel(), cnt.data_ptr(), stream, True)
                    outs.append(out[:int(cnt.item())])
                return torch.cat(outs)
            us, h = timed(run_mfma, args.reps)
            rec["verify_mfma_us"] = round(us, 1)
            vh["mfma"] = torch.sort(h).values.cpu()
        for k, v in vh.items():
            rec[f"verify_{k}_hits"] = int(v.numel())
        if len(vh) == 2:
            rec["verify_agree"] = bool(torch.equal(vh["bpg"], vh["mfma"]))
        rec["verify_pairs"] = int(pairs.numel())
        print(json.dumps(rec), flush=True)


def library_ab(args):
    """The production question: which of the bench library's BPG programs could the MFMA engine
    take at all (<= 64 byte-level positions, no code-point contexts: fits_group), and where it can,
    which engine is faster on the bench's own log text (request-sized candidate verify, bulk
    verify of every candidate line, literal-free scan of every line)."""
    from log_parser_amd.utils.synth import make_log, realistic_library
    dev = torch.device("cuda", 0)
    sets, trig = realistic_library(1000, seed=7)
    full = CompiledLibrary(sets, ScoringParams())
    blob = make_log(250_000, trig, seed=11, hit_rate=0.05, aux_rate=0.01, stack_rate=0.01).encode()
    reps = max(1, args.lines // (blob.count(b"\n") + 1))
    data = b"\n".join([blob] * reps)
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(dev)
    ls, ll = K.split_lines(t, len(data))
    L = ls.numel()
    stream = torch.cuda.current_stream().cuda_stream
    rng = random.Random(7)
    summary = {"library_bpg_programs": len(full.bpg_regs), "mfma_runnable": 0, "lines": L}
    for r in full.bpg_regs:
        pat = full.regexes[r].pattern
        d = N.compile_regex(pat, 4, 4096)
        rec = {"regex": pat, "bpg_words": int(np.frombuffer(N.compile_regex(pat)["bpg"], np.uint64)[0] & np.uint64(0xFF))
               if N.compile_regex(pat)["bpg"] else None, "byte_positions": int(d["npos"]), "cp_only": bool(d["cp_only"])}
        if not fits_group(d):
            rec["mfma"] = ("code-point contexts (no byte NFA)" if d["cp_only"] or not d["npos"]
                           else f"{int(d['npos'])} byte positions > 64 per MFMA group")
            print(json.dumps(rec), flush=True)
            continue
        summary["mfma_runnable"] += 1
        ps = PatternSet.model_validate({"metadata": {"library_id": "one"}, "patterns": [
            {"id": "p", "name": pat, "severity": "HIGH", "primary_pattern": {"regex": pat, "confidence": 0.5}}]})
        lib = CompiledLibrary([ps], ScoringParams(), max_dfa_states=4)
        groups = pack_groups([(lib.bpg_regs[0], d)])
        tabs_np, ncls = zip(*[build_group(g) for g in groups])
        gt = torch.from_numpy(np.concatenate(tabs_np).view(np.int64)).to(dev)
        gl = torch.zeros(1, dtype=torch.int32, device=dev)
        btabs = lib.device_tables(dev)
        regs = torch.tensor(lib.bpg_regs, dtype=torch.int32, device=dev)
        cap = max(4096, L // 2)
        us_b, hb = timed(lambda: K.scan(t, ls, ll, regs, btabs["dfa"], cap), args.reps)
        us_m, hm = timed(lambda: K.nfa_scan(gt, gl, ncls[0], t, ls, ll, cap), args.reps)
        rec.update(scan_bpg_us=round(us_b, 1), scan_mfma_us=round(us_m, 1),
                   scan_agree=bool(torch.equal(torch.sort(hb).values.cpu(), torch.sort(hm).values.cpu())))
        for name, C in (("request", min(200, L)), ("bulk", min(args.cands, L))):
            lines = torch.tensor(sorted(rng.sample(range(L), C)), dtype=torch.int32, device=dev)
            pairs = regs.to(torch.int64)[:, None] << 32 | lines.to(torch.int64)[None, :]
            pairs = pairs.reshape(-1)

            def run_bpg():
                c = pairs.clone()
                N.bpg_cand_dev(c.data_ptr(), c.numel(), t.data_ptr(), ls.data_ptr(), ll.data_ptr(), btabs["dfa"], stream)
                return c[c >= 0]

            def run_mfma():
                out = torch.empty(C + 1, dtype=torch.int64, device=dev)
                cnt = torch.zeros(1, dtype=torch.int64, device=dev)
                N.nfa(gt.data_ptr(), gl.data_ptr(), 1, ncls[0], lines.data_ptr(), C, t.data_ptr(), ls.data_ptr(),
                      ll.data_ptr(), 0, out.data_ptr(), out.numel(), cnt.data_ptr(), stream, True)
                return out[:int(cnt.item())]
            ub, vb = timed(run_bpg, args.reps)
            um, vm = timed(run_mfma, args.reps)
            rec.update({f"verify_{name}_bpg_us": round(ub, 1), f"verify_{name}_mfma_us": round(um, 1),
                        f"verify_{name}_agree": bool(torch.equal(torch.sort(vb).values.cpu(), torch.sort(vm).values.cpu()))})
        print(json.dumps(rec), flush=True)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
