"""LDS bank-conflict model of k_scan_multi's hot walk (scan_multi.hip) on the bench's library and log.

Emulates the bulk variant: one lane walks a run of 4 lines from the 16-byte block holding the run's
first byte to its last separator, 64 consecutive runs per wave, all lanes in lock step. For every
per-group row read (ds_read_u16 at row + bytemap byte) it counts the LDS cycles of the two 32-lane
halves: per bank, the number of DISTINCT dwords the active lanes read (identical addresses
broadcast). Prints cycles per wave-instruction (2 = conflict-free), the state-visit histogram, and
the same model for a renumbering of the non-accepting states by visit frequency.
python tools/scan_bank_sim.py [--waves 40]"""
import argparse
import sys

import numpy as np

sys.path.insert(0, ".")
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.utils.config import ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_log, realistic_library  # noqa: E402


def lds_cycles(addr_bytes, active):
    """cycles of one wave-wide ds_read_u16: two halves of 32 lanes, bank = dword mod 32"""
    cyc = 0
    for h in (slice(0, 32), slice(32, 64)):
        a = addr_bytes[h][active[h]] >> 2
        if a.size == 0:
            continue
        d = np.unique(a)
        cyc += np.bincount(d % 32, minlength=32).max()
    return cyc


def simulate(blob16, sp, g, text, starts, ends, waves, run_len=4):
    rb, init = sp["row_base"][g], sp["init_row"][g]
    bm = np.frombuffer(np.asarray(sp["blob"][:256], np.uint32).tobytes(), np.uint32)
    col2 = ((bm >> np.uint32(8 * g)) & np.uint32(0xFF)).astype(np.int64)
    nl = len(starts)
    tot_cyc = tot_ins = 0
    visits = {}
    for w in range(waves):
        r0 = w * 64 * run_len * 7 % max(1, nl - 64 * run_len)
        lo = np.array([starts[min(r0 + k * run_len, nl - 1)] for k in range(64)])
        hi = np.array([ends[min(r0 + k * run_len + run_len - 1, nl - 1)] + 1 for k in range(64)])
        pos = lo & ~15
        xr = np.full(64, init, np.int64)
        steps = int((hi - pos).max())
        for s in range(steps):
            p = pos + s
            act = p < hi
            c = text[np.minimum(p, len(text) - 1)].astype(np.int64)
            addr = xr + col2[c]
            tot_cyc += lds_cycles(addr, act)
            tot_ins += 1
            for st in ((xr[act] - rb) // (2 * sp["stride"][g])).tolist():
                visits[st] = visits.get(st, 0) + 1
            nxt = blob16[addr >> 1].astype(np.int64)
            xr = np.where(act, nxt, xr)
    return tot_cyc / max(tot_ins, 1), visits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=40)
    ap.add_argument("--patterns", type=int, default=1000)
    a = ap.parse_args()
    sets, trig = realistic_library(a.patterns, seed=7)
    lib = CompiledLibrary(sets, ScoringParams())
    sp = lib.scan_passes[0]
    blob = np.asarray(sp["blob"], np.uint32)
    blob16 = blob[:sp["lds_words"]].view(np.uint16)
    text = np.frombuffer(make_log(40000, trig, seed=11, hit_rate=0.004, aux_rate=0.01,
                                  stack_rate=0.01).encode(), np.uint8)
    nlp = np.flatnonzero(text == 10)
    starts = np.concatenate([[0], nlp[:-1] + 1])
    ends = nlp                                        # the separator of each line
    for g in range(sp["ngroups"]):
        cyc, visits = simulate(blob16, sp, g, text, starts, ends, a.waves)
        v = sorted(visits.items(), key=lambda kv: -kv[1])
        tot = sum(visits.values())
        top = [(s, round(n / tot, 3)) for s, n in v[:8]]
        print(f"group {g}: {cyc:.2f} LDS cycles per row read (2 = conflict-free); states visited "
              f"{len(visits)}; top states {top}")


if __name__ == "__main__":
    main()
