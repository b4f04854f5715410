"""Per-op GPU times of the single-request path (10k lines, 1k patterns): each native op timed in
isolation with HIP events (warm caches, 50 reps), to separate kernel latency from launch/sync
overhead in the /parse p50."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from log_parser_amd.engine import Engine, Segments  # noqa: E402
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.ops import kernels as K  # noqa: E402
from log_parser_amd.utils.config import Config, ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_library, make_log  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 1)


def main():
    dev = torch.device("cuda", 0)
    lines = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    sets, trig = make_library(1000, seed=7)
    lib = CompiledLibrary(sets, ScoringParams())
    eng = Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
    data = make_log(lines, trig, seed=13, hit_rate=0.01).encode()
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    t = t.to(dev)
    n = len(data)
    ls, ll = K.split_lines(t, n)
    L = ls.numel()
    segs = Segments.single(L, dev)
    evt = eng._ev_tables(segs)
    tabs = eng.tabs
    out = {"lines": L}
    out["empty_kernel_fill"] = timeit(lambda: torch.zeros(1, device=dev))
    out["blk_index"] = timeit(lambda: K.line_block_index(ls, n))
    blk = K.line_block_index(ls, n)
    gh = torch.empty(1 << 22, dtype=torch.int64, device=dev)
    cand = torch.empty(1 << 22, dtype=torch.int64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    from log_parser_amd.native import N
    s = torch.cuda.current_stream().cuda_stream

    def pf():
        cnt.zero_()
        N.prefilter_dev(t.data_ptr(), n, tabs["pf"], ls.data_ptr(), L, gh.data_ptr(), 1 << 22, cnt.data_ptr(),
                        eng.pf_grid, s)

    def pfv(grid):
        cnt[1:].zero_()
        N.pf_verify_dev(gh.data_ptr(), 1 << 22, t.data_ptr(), n, tabs["pf"], ls.data_ptr(), L, blk.data_ptr(),
                        cand.data_ptr(), 1 << 22, cnt.data_ptr() + 8, s, cnt.data_ptr(), grid)
    out["prefilter"] = timeit(pf)
    pf()
    for g in (16, 128, 1024):
        out[f"pf_verify_grid{g}"] = timeit(lambda: pfv(g))
    pfv(128)
    c = cnt.cpu().tolist()
    out["gram_hits"], out["candidates"] = c
    cands, pre = eng.match_candidates(t, n, ls, ll)
    out["post_hits"] = timeit(lambda: K.post_hits(cands, pre, L, lib.n_regexes, t, ls, ll, tabs["dfa"], evt, eng.ws))
    hits, hit_line, hit_off, ev_cnt, ev_end, nh, ne = K.post_hits(cands, pre, L, lib.n_regexes, t, ls, ll,
                                                                  tabs["dfa"], evt, eng.ws)
    out["hits"], out["events"] = nh, ne
    ext = lib.ctx_dfa_extent
    out["post_events"] = timeit(lambda: K.post_events(hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll, tabs["dfa"],
                                                      len(lib.freq_ids), eng.ws, ctx_ext=ext))
    out["post_events_nofeat"] = timeit(lambda: K.post_events(hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll,
                                                             tabs["dfa"], len(lib.freq_ids), eng.ws, features=False))
    *_, cov = K.post_events(hits, nh, ev_cnt, ev_end, ne, L, evt, t, ls, ll, tabs["dfa"], len(lib.freq_ids), eng.ws,
                            features=False)
    covered = torch.nonzero(cov[:L] > 0).flatten().to(torch.int32)
    out["covered_lines"] = covered.numel()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
