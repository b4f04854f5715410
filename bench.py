#!/usr/bin/env python3
"""Headline benchmark: log-lines/sec parsed+scored (whole node), 1k-pattern library.

Config (BASELINE.json configs[2], weak-scaled): every rank (one process per GPU) owns a shard of
``--lines-per-gpu`` lines (default 12.5M -> 100M lines on 8 GPUs) of one logical synthetic pod
log, analysed against a randomly generated 1,000-pattern library (primary + secondary +
sequence patterns, context rules). A timed step is the complete pipeline for the shard:

  pinned host -> HBM copy of the raw log bytes (PCIe ingest, H2D)
  -> line index -> literal prefilter -> DFA verify / scan -> hit CSR -> events
  -> packed RCCL all_gather (global N, frequency carry, sequence-chain carry)
  -> fused fp64 scoring -> RCCL all_reduce (severity + frequency histograms)
  -> RCCL all_gather top-k -> persistent frequency-state update.

Nothing is cached between steps (the frequency state evolves exactly as the reference's would).
Rank 0 prints one JSON line; ``value`` is total lines/s over all ranks (max step time across
ranks). The reference publishes no number, so ``vs_baseline`` is null.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lines-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--block-lines", type=int, default=250_000, help="unique synthetic lines, tiled to the shard")
    ap.add_argument("--hit-rate", type=float, default=0.004)
    ap.add_argument("--topk", type=int, default=100)
    ap.add_argument("--profile", action="store_true", help="per-stage HIP-event timings (no extra syncs)")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--parse-requests", type=int, default=30,
                    help="rank 0: p50 latency of N single 10k-line /parse requests after the timed loop (0 = off)")
    ap.add_argument("--torch-trace", default="", help="after timing, run one step under torch.profiler -> chrome trace")
    ap.add_argument("--no-overlap", action="store_true", help="serialise H2D ingest with compute")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend: auto = nccl (RCCL) on GPUs; gloo = host-staged collectives, "
                         "only to rehearse several ranks on ONE GPU")
    return ap.parse_args()


def main():
    args = parse()
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.parallel.dp import ShardedAnalyzer
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils import tracing as TR
    from log_parser_amd.utils.synth import make_library, make_log

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and args.device != "cpu"
    if use_cuda:
        local_gpu = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_gpu)
        device = torch.device("cuda", local_gpu)
        from log_parser_amd.utils.numa import bind_to_gpu_numa
        bind_to_gpu_numa(local_gpu)          # pinned ingest buffers on the GPU's own socket
    else:
        device = torch.device("cpu")
    if world > 1:
        backend = args.backend if args.backend != "auto" else ("nccl" if use_cuda else "gloo")
        dist.init_process_group(backend, rank=rank, world_size=world)

    params = ScoringParams()
    sets, trig = make_library(args.patterns, seed=7)
    lib = CompiledLibrary(sets, params)
    cfg = Config.load(overrides={"engine.device": str(device)})
    eng = Engine(lib, cfg, device=device)
    eng.profile = args.profile
    sa = ShardedAnalyzer(eng)

    # ---- synthetic shard: block tiled to lines_per_gpu, plus halo lines from the neighbours
    block = make_log(args.block_lines, trig, seed=11, hit_rate=args.hit_rate, aux_rate=0.01, stack_rate=0.01)
    block_b = block.encode()
    blines = block_b.split(b"\n")[:-1]
    reps = max(1, args.lines_per_gpu // len(blines))
    own = block_b * reps
    own_lines = len(blines) * reps
    H = lib.halo
    head = b"\n".join(blines[:H]) + b"\n"
    tail = b"\n".join(blines[-H:]) + b"\n"
    hl = H if rank > 0 else 0
    hr = H if rank < world - 1 else 0
    data = (tail if hl else b"") + own + (head if hr else b"")
    nbytes = len(data)
    size = K.padded_len(nbytes)
    host = torch.zeros(size, dtype=torch.uint8, pin_memory=use_cuda)
    host[:nbytes].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    del data, own
    # Double-buffered ingest: the PCIe copy of request k+1 runs on its own HIP stream while request
    # k is analysed (every step still moves all of its bytes host->HBM). --no-overlap serialises.
    bufs = [torch.empty(size, dtype=torch.uint8, device=device) for _ in range(2)]
    copy_stream = torch.cuda.Stream(device) if use_cuda else None
    ready = [torch.cuda.Event() for _ in range(2)] if use_cuda else None
    free = [torch.cuda.Event() for _ in range(2)] if use_cuda else None
    freed = [False, False]
    state = {"i": 0, "issued": -1}

    def issue_copy(i):
        b = i % 2
        if not use_cuda:
            bufs[b].copy_(host)
            return
        with torch.cuda.stream(copy_stream):
            if freed[b]:
                copy_stream.wait_event(free[b])
            bufs[b].copy_(host, non_blocking=True)
            ready[b].record(copy_stream)
        state["issued"] = i

    def step():
        i = state["i"]
        b = i % 2
        if state["issued"] < i:
            issue_copy(i)
        if use_cuda:
            torch.cuda.current_stream().wait_event(ready[b])
        if not args.no_overlap:
            issue_copy(i + 1)                                    # prefetch the next request
        text = bufs[b]
        if use_cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        ls, ll = K.split_lines(text, nbytes)
        out = sa.step(text, nbytes, ls, ll, hl, hr, topk=args.topk)
        if use_cuda:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            state.setdefault("dev", []).append((ev0, ev1))
        if rank == 0 and out.topk_score is not None:
            out.topk_score.cpu()                                 # results land on the host
        if use_cuda:
            free[b].record(torch.cuda.current_stream())
            freed[b] = True
        state["i"] = i + 1
        return out

    def barrier():
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    state["dev"] = []
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step()
    barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=device)
    if world > 1:
        if dist.get_backend() == "gloo":
            dt_t = dt_t.cpu()
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_lines = last.total_lines
    ms = dt / args.steps * 1e3
    value = total_lines * args.steps / dt
    if rank == 0:
        rec = {
            "metric": "log-lines/sec parsed+scored (whole node), 1k-pattern library",
            "value": round(value, 1), "unit": "lines/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp64", "data": "synthetic",
            "ingest": "h2d-serial" if args.no_overlap else "h2d-overlapped(2 buffers, copy stream)",
            "config": {"model": f"log-parser {args.patterns}-pattern random library (secondary+sequence+context)",
                       "global_batch": total_lines, "seq_len": round(nbytes / max(own_lines, 1), 1),
                       "parallelism": f"dp{world}", "lines_per_gpu": own_lines, "bytes_per_gpu": nbytes,
                       "events_per_step": int(last.pattern_counts.sum().item()),
                       "library": lib.summary(), "device": str(device)},
        }
        if state.get("dev"):
            # compute-stream time of the device pipeline per step (line index .. collectives .. top-k),
            # i.e. what the GPU sustains when the log is already resident (the timed value above
            # includes every byte's PCIe copy, overlapped on the copy stream)
            dms = float(np.mean([a.elapsed_time(b) for a, b in state["dev"]]))
            rec["device_ms_per_step_rank0"] = round(dms, 3)
            rec["device_resident_lines_per_s"] = round(own_lines * world / (dms / 1e3), 1)
        if args.profile:
            rec["timings_ms_last_step_rank0"] = {k: round(v, 3) for k, v in TR.resolve(last.result.timings).items()}
        if args.parse_requests > 0:
            # second half of the BASELINE metric: p50 latency of one /parse request (10k-line pod
            # log, same 1k-pattern library) through the serving engine path (staging, kernels,
            # JSON). Measured after the timed loop, outside it; HTTP framing excluded.
            req = make_log(10_000, trig, seed=13, hit_rate=0.01)
            for _ in range(3):
                eng.analyze_batch_json([req])
            lat = []
            for _ in range(args.parse_requests):
                t1 = time.perf_counter()
                eng.analyze_batch_json([req])
                lat.append(time.perf_counter() - t1)
            rec["p50_parse_ms"] = round(float(np.median(lat)) * 1e3, 3)
            rec["p99_parse_ms"] = round(float(np.percentile(lat, 99)) * 1e3, 3)
            rec["config"]["parse_request_lines"] = 10_000
        print(json.dumps(rec), flush=True)
    if args.torch_trace:                                         # untimed, after the measurement
        with TR.torch_profile(args.torch_trace.replace(".json", f".rank{rank}.json"), device):
            step()
            barrier()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
