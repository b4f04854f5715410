#!/usr/bin/env python3
"""Headline benchmark: log-lines/sec parsed+scored (whole node), 1k-pattern library; p50 /parse.

Config (BASELINE.json configs[2], weak-scaled): every rank (one process per GPU) owns a shard of
``--lines-per-gpu`` lines (default 12.5M -> 100M lines on 8 GPUs) of one logical synthetic pod
log, analysed against a randomly generated 1,000-pattern library (primary + secondary +
sequence patterns, context rules; ``--library realistic`` adds 3-6-byte-literal and literal-free
primaries). A timed step is the complete pipeline for the shard:

  pinned host -> HBM copy of the raw log bytes (PCIe ingest, H2D)
  -> line index -> literal prefilter -> DFA verify / scan -> hit CSR -> events
  -> collective 1: packed in-place RCCL all_gather (global N, frequency carry, sequence-chain
     carry, overflow veto)
  -> fused fp64 scoring -> summary kernel
  -> collective 2: in-place RCCL all_gather of [pattern + severity histograms | frequency counts |
     top-k rows], summed / merged locally (~20 KB per rank: one all_gather instead of an
     all_reduce + an all_gather) -> persistent frequency-state update
  -> every event record (line, pattern, score) copied to pinned host memory.

Launch: ``python bench.py --gpus N`` starts N rank processes itself (``utils/launch.py``; the
parent makes no GPU call) -- or runs as one rank of ``torch.distributed.run``. On GPUs the
process group is ``nccl`` (= RCCL over xGMI) at every world size, including 1: the 1-GPU number
runs the same two in-place all-gathers per step as the 8-GPU run (``parallel/dp.py``).

Nothing is cached between steps (the frequency state evolves exactly as the reference's would).
Rank 0 prints one JSON line; ``value`` is total lines/s over all ranks (max step time across
ranks). The reference publishes no number, so ``vs_baseline`` is null. After the
timed loop rank 0 measures p50/p99 of ``POST /parse`` (10k-line body) through a real server
process started before this process touched the GPU (``p50_parse_ms``), and the engine-only
latency of the same request (``p50_engine_ms``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "log-lines/sec parsed+scored (whole node), 1k-pattern library"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lines-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--library", default="realistic", choices=["realistic", "synthetic"],
                    help="realistic: ~10%% short-literal and ~5%% literal-free primaries; synthetic: every "
                         "primary has a long unique literal (the prefilter's best case)")
    ap.add_argument("--block-lines", type=int, default=250_000, help="lines of one generated synthetic block")
    ap.add_argument("--distinct-blocks", type=int, default=4,
                    help="distinct generated blocks (seeds); the shard tiles them in rotation, rank r starting at "
                         "block r, so hit / candidate distributions do not repeat one block")
    ap.add_argument("--hit-rate", type=float, default=0.004)
    ap.add_argument("--topk", type=int, default=100)
    ap.add_argument("--profile", action="store_true", help="per-stage HIP-event timings (no extra syncs)")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--parse-requests", type=int, default=300,
                    help="rank 0: p50 latency of N single 10k-line POST /parse requests after the timed loop (0 = off)")
    ap.add_argument("--http", default="native", choices=["native", "uvicorn"], help="server front end for p50")
    ap.add_argument("--server-env", action="append", default=[], metavar="KEY=VALUE",
                    help="extra environment of the /parse server process only (A/B knob, repeatable)")
    ap.add_argument("--torch-trace", default="", help="after timing, run one step under torch.profiler -> chrome trace")
    ap.add_argument("--no-overlap", action="store_true", help="serialise H2D ingest with compute")
    ap.add_argument("--pf-verify-lanes", type=int, default=0, choices=[0, 1, 2, 4, 16],
                    help="A/B: lanes per gram hit in the bulk literal verify (0: the kernel's default)")
    ap.add_argument("--scan-defer-rare", type=int, default=1, choices=[0, 1],
                    help="A/B: the scan walk's hot blocks re-walked by k_scan_rare (1) or inline (0)")
    ap.add_argument("--d2h-stream", default="copy", choices=["copy", "compute"],
                    help="stream of the per-step event D2H (diagnostic A/B)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo", "none"],
                    help="process group: auto = nccl (RCCL) on GPUs at every world size, gloo on CPU for world "
                         "size > 1 and none on CPU at world size 1; nccl / gloo / none force one (gloo on GPUs "
                         "= host-staged, to rehearse several ranks on ONE GPU; none = no collectives at world 1)")
    ap.add_argument("--counted-repeats", type=int, default=0,
                    help="add N primaries with a wide bounded repeat (X.{0,2100}Y, X[^;]{0,5000}Y, X\\S{0,20000}Y): "
                         "counted BPG positions")
    ap.add_argument("--bt-patterns", type=int, default=0,
                    help="add N primaries only a backtracker decides (backreference / lookaround / atomic; N-1 with "
                         "a literal, one literal-free): the device feeds them with their relaxed automata and the host "
                         "checks only the candidate lines, inside the queued step (side_path.hip)")
    ap.add_argument("--lookaround-patterns", type=int, default=0,
                    help="add N primaries with lookaround line filters (X(?!ure), (?<!retrying )X, X(?!.*retry), "
                         "(?=.*FATAL)X, (?<!\\S)X(?!\\S)): exact find() DFAs, no backtracker")
    ap.add_argument("--ranks-per-gpu", type=int, default=1,
                    help="REHEARSAL of a multi-GPU run on fewer GPUs: --gpus N ranks share N / R GPUs (R ranks "
                         "each), with gloo (host-staged) collectives -- RCCL takes one rank per GPU. Same spawn, "
                         "heartbeats, shards, halos and both collectives as the N-GPU run; n_gpus reports N / R")
    ap.add_argument("--gen-workers", type=int, default=4,
                    help="forked processes generating the synthetic blocks (0: in this process -- under "
                         "rocprofv3 --pmc, whose preloaded library has initialised the GPU before main)")
    ap.add_argument("--phase-log", default="",
                    help="append every rank's phases (JSON lines) to PATH.rank<r>.jsonl")
    ap.add_argument("--timeout", type=float, default=1500.0,
                    help="hang guard: the whole job's deadline in seconds (0 = none)")
    ap.add_argument("--stall-timeout", type=float, default=300.0,
                    help="hang guard: seconds without ANY rank advancing a phase (utils/heartbeat.py); on expiry "
                         "rank 0 prints one JSON line with status 'timeout' and every rank's last phase")
    ap.add_argument("--pg-timeout", type=float, default=300.0, help="init_process_group / collective timeout (s)")
    return ap.parse_args()


def _gen_block(job):
    """One synthetic block (forked pool worker: no GPU state exists yet)."""
    trig, n, seed, hit_rate = job
    from log_parser_amd.utils.synth import make_log
    return make_log(n, trig, seed=seed, hit_rate=hit_rate, aux_rate=0.01, stack_rate=0.01).encode()


def make_blocks(args, trig):
    """``--distinct-blocks`` blocks of ``--block-lines`` lines, generated in parallel BEFORE any GPU
    call (forking after HIP initialisation is not allowed)."""
    jobs = [(trig, args.block_lines, 11 + 7919 * b, args.hit_rate) for b in range(max(1, args.distinct_blocks))]
    if len(jobs) == 1 or args.gen_workers <= 0:
        return [_gen_block(j) for j in jobs]
    import multiprocessing as mp
    with mp.get_context("fork").Pool(min(len(jobs), args.gen_workers)) as pool:
        return pool.map(_gen_block, jobs)


def library(args):
    from log_parser_amd.utils.synth import (backtracker_patterns, counted_repeat_patterns, lookaround_patterns,
                                            make_library, realistic_library)
    if args.library == "realistic":
        sets, trig = realistic_library(args.patterns, seed=7)
    else:
        sets, trig = make_library(args.patterns, seed=7)
    if args.bt_patterns > 0:
        ps, bt_trig = backtracker_patterns(args.bt_patterns, seed=7)
        sets, trig = sets + [ps], trig + bt_trig
    if args.counted_repeats > 0:
        ps, cr_trig = counted_repeat_patterns(args.counted_repeats, seed=7)
        sets, trig = sets + [ps], trig + cr_trig
    if args.lookaround_patterns > 0:
        ps, la_trig = lookaround_patterns(args.lookaround_patterns, seed=7)
        sets, trig = sets + [ps], trig + la_trig
    return sets, trig


def _digest(out, top) -> str:
    """sha256 (16 hex) of a step's global results: pattern / severity / frequency histograms and the
    merged top-k rows -- equal for any world size over the same concatenated log."""
    if out is None:
        return ""
    import hashlib
    h = hashlib.sha256()
    for t in (out.pattern_counts, out.severity_counts, out.freq_counts, top):
        if t is not None:
            h.update(t.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:16]


def main():
    args = parse()
    from log_parser_amd.utils import launch
    # >= 8 HIP hardware queues, before any HIP call here, in the ranks or in the /parse server: with
    # HIP's default 4 an RCCL group's streams push the ingest copy onto a kernel queue and the copy
    # stops overlapping the step (23.5 -> 27.1 ms/step at world 1, profiles/r3_f)
    hw_queues = launch.ensure_hw_queues()
    if not launch.under_launcher() and args.gpus > 1:
        # parent: no GPU call here; N fresh rank processes, one per GPU, under the same hang guard
        sys.exit(launch.spawn_local_ranks([os.path.abspath(__file__)] + sys.argv[1:], args.gpus,
                                          timeout_s=(args.timeout + 60) if args.timeout else None,
                                          stall_s=(args.stall_timeout + 60) if args.stall_timeout else None,
                                          metric=METRIC))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from log_parser_amd.utils.heartbeat import Heartbeat
    hb = Heartbeat(rank, world, log_path=args.phase_log)
    hb.start(METRIC, args.stall_timeout, args.timeout or None)
    sets, trig = library(args)
    hb.phase("library")
    blocks = make_blocks(args, trig)
    hb.phase("blocks")

    # p50 /parse server: started BEFORE this process makes any GPU call (rank 0 only)
    server = None
    if rank == 0 and args.parse_requests > 0:
        from log_parser_amd.utils import restbench
        dev = "cpu" if args.device == "cpu" else f"cuda:{local_rank}"
        server = restbench.ServerProcess(restbench.write_library(sets), dev, http=args.http,
                                         env=dict(kv.split("=", 1) for kv in args.server_env))
    try:
        run(args, sets, trig, blocks, rank, world, local_rank, server, hw_queues, hb)
    finally:
        if server is not None:
            server.stop()
        hb.phase("done")
        hb.stop()


def run(args, sets, trig, blocks, rank, world, local_rank, server, hw_queues=0, hb=None):
    import numpy as np
    import torch
    import torch.distributed as dist
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.ops import kernels as K
    from log_parser_amd.parallel.dp import ShardedAnalyzer, all_gather_rows
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils import tracing as TR
    from log_parser_amd.utils import launch
    from log_parser_amd.utils.synth import make_log

    use_cuda = torch.cuda.is_available() and args.device != "cpu"
    if use_cuda:
        ngpu = torch.cuda.device_count()
        rpg = max(1, args.ranks_per_gpu)
        if world > ngpu * rpg:
            raise SystemExit(f"{world} ranks but {ngpu} visible GPU(s) x {rpg} rank(s) per GPU "
                             f"(a rehearsal on fewer GPUs: --ranks-per-gpu)")
        local_gpu = local_rank // rpg
        torch.cuda.set_device(local_gpu)
        device = torch.device("cuda", local_gpu)
        # the ingest copy stream is created before RCCL creates its own: HIP maps streams to a few
        # hardware queues in creation order (GPU_MAX_HW_QUEUES), and a copy stream created after the
        # process group can share the compute stream's queue -- the copy then waits for the step's
        # kernels instead of overlapping them (profiles/r3_f)
        early_copy_stream = torch.cuda.Stream(device)
        from log_parser_amd.utils.numa import bind_to_gpu_numa
        bind_to_gpu_numa(local_gpu)          # pinned ingest buffers on the GPU's own socket
    else:
        device = torch.device("cpu")
        early_copy_stream = None
    backend = args.backend
    if backend == "auto":
        # GPUs: RCCL at every world size, 1 included -- the 1-GPU number runs the same collectives as
        # the 8-GPU one (with >= 8 HW queues the world-1 group costs nothing, profiles/r3_f)
        backend = "nccl" if use_cuda else ("gloo" if world > 1 else "none")
    if backend == "none" and world > 1:
        backend = "nccl" if use_cuda else "gloo"
    if args.ranks_per_gpu > 1 and backend == "nccl":
        backend = "gloo"                    # RCCL: one rank per GPU; the rehearsal stages through the host
    if backend != "none":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            from log_parser_amd.utils.launch import free_port
            os.environ["MASTER_PORT"] = str(free_port())
        kw = {"device_id": device} if backend == "nccl" else {}
        from datetime import timedelta
        from log_parser_amd.utils.launch import stdout_to_stderr
        hb.phase("init_process_group")
        with stdout_to_stderr():            # RCCL prints its version banner on stdout: keep ONE JSON line
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=timedelta(seconds=args.pg_timeout),
                                    **kw)
            hb.phase("first barrier")
            dist.barrier()
        hb.phase("process group ready")
        assert dist.get_world_size() == world

    from log_parser_amd.native import N
    if args.pf_verify_lanes:
        N.set_pf_verify_lanes(args.pf_verify_lanes)
    N.set_scan_defer_rare(bool(args.scan_defer_rare))
    params = ScoringParams()
    lib = CompiledLibrary(sets, params)
    cfg = Config.load(overrides={"engine.device": str(device)})
    eng = Engine(lib, cfg, device=device)
    eng.profile = args.profile
    sa = ShardedAnalyzer(eng)
    sa.time_reduce = use_cuda and rank == 0        # rank 0's local sum + top-k merge of collective 2 (events)
    hb.phase("engine")

    # ---- synthetic shard: the distinct blocks tiled in rotation to lines_per_gpu (rank r's tiling
    # continues where rank r-1's ends), plus halo lines from the neighbours' adjacent blocks
    B = len(blocks)
    blk_lines = [b.count(b"\n") for b in blocks]
    reps = max(1, args.lines_per_gpu // blk_lines[0])
    order = [(rank * reps + i) % B for i in range(reps)]
    own_lines = sum(blk_lines[j] for j in order)
    H = lib.halo

    def edge(b, first):
        ls_ = blocks[b].split(b"\n", H) if first else blocks[b][:-1].rsplit(b"\n", H)
        return b"\n".join(ls_[:H] if first else ls_[-H:]) + b"\n"
    hl = H if rank > 0 else 0
    hr = H if rank < world - 1 else 0
    pre = edge(((rank - 1) * reps + reps - 1) % B, False) if hl else b""
    post = edge(((rank + 1) * reps) % B, True) if hr else b""
    parts = [pre] + [blocks[j] for j in order] + [post]
    nbytes = sum(len(x) for x in parts)
    size = K.padded_len(nbytes)
    # page-locked host shard, registered in place (utils/hostmem.py); the H2D is an SDMA copy
    if use_cuda:
        from log_parser_amd.utils.hostmem import registered_empty
        host = registered_empty(size)
        host.zero_()
    else:
        host = torch.zeros(size, dtype=torch.uint8)
    hv = host.numpy()
    o = 0
    for part in parts:                                     # fill in place: no whole-shard temporaries
        hv[o:o + len(part)] = np.frombuffer(part, np.uint8)
        o += len(part)
    # Double-buffered ingest: the PCIe copy of request k+1 runs on its own HIP stream while request
    # k is analysed (every step still moves all of its bytes host->HBM). --no-overlap serialises.
    bufs = [torch.empty(size, dtype=torch.uint8, device=device) for _ in range(2)]
    copy_stream = (early_copy_stream or torch.cuda.Stream(device)) if use_cuda else None
    ready = [torch.cuda.Event() for _ in range(2)] if use_cuda else None
    free = [torch.cuda.Event() for _ in range(2)] if use_cuda else None
    freed = [False, False]
    state = {"i": 0, "issued": -1, "events_host": 0}
    # event records land here (pinned, 2 slots so step k+1's copy never waits on step k's)
    ev_host = [torch.empty(0, dtype=torch.uint8, pin_memory=use_cuda) for _ in range(2)]

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

    def events_to_host(out, slot):
        """(global line int64, pattern int32, score f64) of EVERY event -> pinned host, one copy.
        The D2H runs on the copy stream, behind the prefetch H2D: on the compute stream it would
        queue behind the 23 ms PCIe ingest of the next step and stall the next step's kernels."""
        n = out.result.ev_line.numel()
        if n == 0:
            return
        pk = out.events_packed                  # packed by the summary kernel: [line i64 | score f64 | pat i32]
        nb = pk.numel()
        if ev_host[slot].numel() < nb:
            if use_cuda:
                torch.cuda.current_stream().synchronize()        # the old slot may still be in flight
            ev_host[slot] = torch.empty(nb * 5 // 4, dtype=torch.uint8, pin_memory=use_cuda)
        if use_cuda and args.d2h_stream == "copy":
            done = torch.cuda.Event()
            done.record()
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_event(done)
                ev_host[slot][:nb].copy_(pk, non_blocking=True)
                pk.record_stream(copy_stream)
        else:
            ev_host[slot][:nb].copy_(pk, non_blocking=use_cuda)
        state["events_host"] = n

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
        # line index + literal prefilter queued before the index's host read (sa.step builds both)
        # host_text: the shard's bytes on the host (the backtracker regexes' candidate lines are checked there)
        out = sa.step(text, nbytes, None, None, hl, hr, topk=args.topk, pack_events=True,
                      host_text=hv[:nbytes] if lib.host_regs else None)
        events_to_host(out, b)                                   # results land on the host
        if rank == 0 and out.topk_rows is not None:
            state["top"] = out.topk_rows.cpu()                   # merged global top-k on the host
        if rank == 0:
            state["last_out"] = out
        if use_cuda:
            # device span: to the step's last kernel (the step records it before its count read)
            ev1 = out.end_event
            if ev1 is None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
            state.setdefault("dev", []).append((ev0, ev1))
            free[b].record(torch.cuda.current_stream())
            freed[b] = True
        state["i"] = i + 1
        return out

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    # per-rank diagnostics: this rank's pinned-host -> HBM bandwidth (one whole-shard copy, untimed)
    # and its GPU's NUMA node, so an 8-GPU result explains itself (a slow socket, a far buffer)
    h2d_gbps = 0.0
    if use_cuda:
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record()
        bufs[0].copy_(host, non_blocking=True)
        b_.record()
        torch.cuda.synchronize()
        h2d_gbps = size / (a_.elapsed_time(b_) / 1e3) / 1e9
    from log_parser_amd.utils.numa import gpu_numa_node
    numa = gpu_numa_node(local_rank) if use_cuda else -1

    hb.phase("shard")
    for k in range(args.warmup):
        launch.inject_fault(rank, k)                            # (tests: LP_FAULT_RANK / _STEP / _MODE)
        step()
        hb.phase(f"warmup {k}")
    barrier()
    hb.phase("server wait")
    if server is not None and not server.wait_ready():      # server idle before timing starts
        print("warning: /parse server did not come up; p50_parse_ms omitted", file=sys.stderr)
        server.stop()
        server = None
    barrier()
    state["dev"] = []
    t0 = time.perf_counter()
    last = None
    for k in range(args.steps):
        launch.inject_fault(rank, args.warmup + k)
        last = step()
        hb.phase(f"timed {k}")
    barrier()
    hb.phase("timed loop done")
    dt = time.perf_counter() - t0
    dms_local = float(np.mean([a.elapsed_time(b) for a, b in state["dev"]])) if state.get("dev") else -1.0
    diag = [dt, h2d_gbps, dms_local, float(numa)]
    per_rank_diag = [diag]
    if dist.is_initialized():
        dt_t = torch.tensor(diag, dtype=torch.float64, device=device)
        if dist.get_backend() == "gloo":
            dt_t = dt_t.cpu()
        per_rank_diag = all_gather_rows(dt_t).cpu().tolist()
    per_rank = [x[0] for x in per_rank_diag]
    dt = max(per_rank)
    total_lines = last.total_lines
    ms = dt / args.steps * 1e3
    value = total_lines * args.steps / dt
    if rank == 0:
        n_gpus = world // max(1, args.ranks_per_gpu) if use_cuda else world
        rec = {
            "metric": METRIC,
            "value": round(value, 1), "unit": "lines/s", "n_gpus": max(1, n_gpus), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp64", "data": "synthetic",
            "ingest": "h2d-serial" if args.no_overlap else "h2d-overlapped(2 buffers, copy stream)",
            "config": {"model": f"log-parser {args.patterns}-pattern {args.library} library "
                                f"(secondary+sequence+context)",
                       "global_batch": total_lines, "seq_len": round(nbytes / max(own_lines, 1), 1),
                       "parallelism": f"dp{world}", "lines_per_gpu": own_lines, "bytes_per_gpu": nbytes,
                       "distinct_blocks": B, "block_lines": args.block_lines,
                       "extra_primaries": {"backtracker": args.bt_patterns, "counted_repeats": args.counted_repeats,
                                           "lookaround": args.lookaround_patterns},
                       "events_per_step": int(last.pattern_counts.sum().item()),
                       "events_to_host_rank0": state["events_host"],
                       "library_kind": args.library, "library": lib.summary(), "prefilter_stride": lib.pf["stride"], "device": str(device)},
            "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": dist.get_backend() if dist.is_initialized() else "none",
            "ms_per_step_per_rank": [round(x / args.steps * 1e3, 3) for x in per_rank],
            "per_rank": [{"rank": r, "ms_per_step": round(x[0] / args.steps * 1e3, 3), "h2d_GBps": round(x[1], 2),
                          "device_ms": round(x[2], 3), "numa_node": int(x[3])} for r, x in enumerate(per_rank_diag)],
            "collectives_per_step": 2 if dist.is_initialized() else 0,
            "hip_hw_queues": hw_queues,
            "matcher_counts_rank0": dict(eng.arena.last),
            "result_digest": _digest(state.get("last_out"), state.get("top")),
        }
        if args.ranks_per_gpu > 1:
            rec["rehearsal"] = (f"{world} ranks on {rec['n_gpus']} GPU(s), {args.ranks_per_gpu} per GPU, "
                                f"{rec['backend']} collectives staged through host memory (readiness, not a scaling point)")
        if sa.reduce_us:
            rec["reduce_merge_us_rank0"] = {"sum_over_ranks": round(float(np.median([a for a, _ in sa.reduce_us])), 1),
                                            "topk_merge": round(float(np.median([b for _, b in sa.reduce_us])), 1),
                                            "rows": world}
        if state.get("dev"):
            # compute-stream time of the device pipeline per step (line index .. collectives .. top-k
            # .. event copy), i.e. what the GPU sustains when the log is already resident (the timed
            # value above includes every byte's PCIe copy, overlapped on the copy stream)
            dms = float(np.mean([a.elapsed_time(b) for a, b in state["dev"]]))
            rec["device_ms_per_step_rank0"] = round(dms, 3)
            rec["device_resident_lines_per_s"] = round(own_lines * world / (dms / 1e3), 1)
        if args.profile:
            rec["timings_ms_last_step_rank0"] = {k: round(v, 3) for k, v in TR.resolve(last.result.timings).items()}
        if args.parse_requests > 0:
            hb.phase("parse latency")
            # second half of the BASELINE metric: one 10k-line /parse request, same library
            req = make_log(10_000, trig, seed=13, hit_rate=0.01)
            if server is not None:
                lat = server.parse_latencies(req, args.parse_requests, warmup=50)   # server idle since start-up
                rec["p50_parse_ms"] = round(float(np.median(lat)) * 1e3, 3)
                rec["p99_parse_ms"] = round(float(np.percentile(lat, 99)) * 1e3, 3)
                rec["parse_transport"] = f"{args.http} HTTP/1.1 keep-alive, server process on 127.0.0.1"
            for _ in range(3):
                eng.analyze_batch_json([req])
            lat = []
            for _ in range(args.parse_requests):
                t1 = time.perf_counter()
                eng.analyze_batch_json([req])
                lat.append(time.perf_counter() - t1)
            rec["p50_engine_ms"] = round(float(np.median(lat)) * 1e3, 3)
            rec["p99_engine_ms"] = round(float(np.percentile(lat, 99)) * 1e3, 3)
            rec["config"]["parse_request_lines"] = 10_000
        print(json.dumps(rec), flush=True)
    if args.torch_trace:                                         # untimed, after the measurement
        with TR.torch_profile(args.torch_trace.replace(".json", f".rank{rank}.json"), device):
            step()
            barrier()
    if dist.is_initialized():
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
