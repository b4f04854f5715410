#!/usr/bin/env python3
"""Benchmarks for the five BASELINE.json configs (the headline is ../bench.py = config 3).

  rest        config 1: 10k-line log, 20 YAML patterns, CPU-only POST /parse (plumbing), p50 latency
  single      config 2: 1M-line log, 256 patterns, 1 GPU (resident and with PCIe ingest)
  stream      config 4: long stream (default 1B lines, scale with --lines), 4k patterns with secondary
              + sequence patterns, chunked through HBM with carries (parallel/stream.py)
  concurrent  config 5: 10k concurrent /parse requests of mixed sizes through the continuous batcher;
              p50 / p99 request latency and aggregate lines/s
  golden      comparator (b) of BASELINE.md: this repo's pure-Python golden model (the reference
              publishes no numbers and no JVM is available here), lines/s on config-1 data

Every mode prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from log_parser_amd import golden  # noqa: E402
from log_parser_amd.engine import Engine, Segments  # noqa: E402
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.ops import kernels as K  # noqa: E402
from log_parser_amd.utils.config import Config, ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_library, make_log  # noqa: E402


def _dev(args):
    if args.device == "auto":
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    else:
        dev = torch.device(args.device)
    if dev.type == "cuda":
        from log_parser_amd.utils.numa import bind_to_gpu_numa
        bind_to_gpu_numa(dev.index or 0)
    return dev


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _engine(n_patterns, dev, seed=7, library="realistic"):
    """Configs 2 / 4 / 5 run on the realistic library (short-literal, literal-free and bounded-gap
    primaries: utils/synth.realistic_library) unless --library synthetic (the prefilter's best case)."""
    from log_parser_amd.utils.synth import realistic_library
    sets, trig = (realistic_library if library == "realistic" else make_library)(n_patterns, seed=seed)
    lib = CompiledLibrary(sets, ScoringParams())
    return Engine(lib, Config.load(overrides={"engine.device": str(dev)}), device=dev), sets, trig


def mode_rest(args):
    _rest(args, 20, "cpu", "rest-10k-lines-20-patterns-cpu")


def mode_rest_gpu(args):
    """Serving latency on the GPU: POST /parse through FastAPI + the continuous batcher, 10k-line
    body, 1k-pattern library (the p50 half of the headline metric, HTTP framing included)."""
    _rest(args, 1000, "cuda:0" if torch.cuda.is_available() else "cpu", "rest-10k-lines-1000-patterns-gpu")


def _rest(args, n_patterns, device, name):
    """Real HTTP: the service runs as its own process (uvicorn, as deployed) on 127.0.0.1 and the
    client keeps one HTTP/1.1 connection open; the timed region is send body -> full response."""
    import http.client
    import socket
    import subprocess
    import tempfile
    import yaml
    sets, trig = make_library(n_patterns, seed=3, n_sets=2)
    d = tempfile.mkdtemp()
    for i, s in enumerate(sets):
        with open(os.path.join(d, f"s{i}.yaml"), "w") as f:
            yaml.safe_dump(s.model_dump(by_alias=True, exclude_none=True), f)
    logs = make_log(10_000, trig, seed=4, hit_rate=0.01)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srv = subprocess.Popen([sys.executable, "-m", "log_parser_amd.serve", f"-Dpattern.directory={d}",
                            f"-Dengine.device={device}", "-Dserver.host=127.0.0.1", f"-Dserver.port={port}",
                            f"-Dserver.http={args.http}"],
                           cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 240
        while True:
            try:
                c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
                c.request("GET", "/ready")
                r = c.getresponse()
                r.read()
                if r.status == 200:
                    break
            except OSError:
                pass
            if time.time() > deadline or srv.poll() is not None:
                raise RuntimeError("server did not come up")
            time.sleep(0.5)
        body = json.dumps({"pod": {"metadata": {"name": "bench"}}, "logs": logs}).encode()
        hdr = {"content-type": "application/json"}

        def post():
            c.request("POST", "/parse", body=body, headers=hdr)
            r = c.getresponse()
            out = r.read()
            assert r.status == 200, out[:200]
            return out
        for _ in range(5):
            post()
        lat = []
        for _ in range(args.requests):
            t = time.perf_counter()
            post()
            lat.append(time.perf_counter() - t)
        c.close()
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
    lat = np.array(lat)
    print(json.dumps({"config": name, "p50_ms": round(float(np.median(lat)) * 1e3, 3),
                      "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3),
                      "lines_per_s": round(10_000 / float(np.median(lat)), 1), "requests": args.requests,
                      "transport": f"{args.http} HTTP front end, HTTP/1.1 keep-alive on 127.0.0.1"}))


def mode_single(args):
    dev = _dev(args)
    eng, _, trig = _engine(256, dev, library=args.library)
    data = make_log(args.lines, trig, seed=5, hit_rate=0.004, aux_rate=0.01, stack_rate=0.01).encode()
    text, n = eng.stage_text(data)
    ls, ll = K.split_lines(text, n)
    segs = Segments.single(ls.numel(), dev)

    def once(resident: bool):
        t = text
        if not resident:
            t, _ = eng.stage_text(data)
        a, b = K.split_lines(t, n)
        res = eng.run(t, n, a, b, segs, eng.freq_carry())
        eng.commit_frequency(res.freq_counts)
        return res

    from log_parser_amd.parallel.dp import ShardedAnalyzer
    sa = ShardedAnalyzer(eng)

    def whole_step(_):
        # the engine's whole-document pipeline (the bulk step at world 1): the line index with the
        # literal prefilter queued behind it before its one host read, matching and events in
        # device-count mode, score, summary + top-k, frequency record, ONE count read at the end
        return sa.step(text, n, None, None, 0, 0, topk=100).result

    out = {"config": f"single-{args.lines}-lines-256-patterns", "device": str(dev), "bytes": n}
    # Engine.run_document last: a kernel trace's last k_nl_count markers then bracket it
    def document(_):
        return eng.run_document(text, n)

    runs = (("resident_run_api", lambda _: once(True)), ("with_h2d_from_pageable", lambda _: once(False)),
            ("resident_bulk_step", whole_step), ("resident", document))
    for label, fn in runs:
        for _ in range(3):
            fn(None)
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = fn(None)
        _sync(dev)
        dt = (time.perf_counter() - t0) / args.steps
        out[label] = {"ms": round(dt * 1e3, 3), "lines_per_s": round(ls.numel() / dt, 1),
                      "events": int(res.score.numel())}
    print(json.dumps(out))


def mode_stream(args):
    from log_parser_amd.parallel.stream import RepeatBuffer, StreamAnalyzer, auto_chunk_bytes
    dev = _dev(args)
    eng, _, trig = _engine(args.patterns, dev, library=args.library)
    block = make_log(200_000, trig, seed=6, hit_rate=0.004, aux_rate=0.01, stack_rate=0.01).encode()
    lines_per_block = block.count(b"\n")
    total = len(block) * max(1, args.lines // lines_per_block)
    src = RepeatBuffer(block, total)
    # the chunk the timed stream will use (auto: from free HBM and the stream length), fixed so the
    # warm-up sizes the pinned pool for it
    chunk = (args.chunk_mb << 20) or auto_chunk_bytes(dev, total)
    sa = StreamAnalyzer(eng, chunk_bytes=chunk, topk=100, keep_events=False)
    # untimed warm-up stream: pinned pool, kernels, and the allocator's full-chunk-size buffers (4
    # chunks of stream: the ramps reach the full chunk size; a first 8 GiB chunk in the timed run
    # otherwise stalled the copy engine 0.2 s on allocations, profiles/r4_b); then a fresh frequency state
    sa.run(RepeatBuffer(block, min(total, 4 * sa.chunk_bytes)))
    eng.freq.reset_all()
    # the log sits in host RAM: page-lock it before the clock (the chunks are then DMA'd from it
    # directly; an unlockable source is staged through pinned buffers inside the timed run)
    src_pinned = dev.type == "cuda" and src.pinned_block() is not None
    _sync(dev)
    t0 = time.perf_counter()
    res = sa.run(src)
    _sync(dev)
    dt = time.perf_counter() - t0
    import hashlib
    digest = hashlib.sha256(np.concatenate([res.topk_score.view(np.int64), res.topk_line,
                                            res.topk_pat]).tobytes()).hexdigest()[:16]
    print(json.dumps({"config": f"stream-{res.total_lines}-lines-{args.patterns}-patterns", "device": str(dev),
                      "seconds": round(dt, 3), "lines_per_s": round(res.total_lines / dt, 1),
                      "bytes": res.bytes, "GB_per_s": round(res.bytes / dt / 1e9, 3), "chunks": res.chunks,
                      "chunk_bytes": sa.chunk_bytes, "events": res.n_events, "summary": res.summary,
                      "source": "page-locked host RAM (direct DMA)" if src_pinned else "host RAM (staged)",
                      "topk_digest": digest}))


def mode_resident(args):
    """A >= 50 GB log kept resident in HBM (parallel/stream.ResidentLog) and analysed twice with two
    different 1k-pattern libraries: the load crosses PCIe once, each re-analysis reads HBM only."""
    from log_parser_amd.parallel.stream import RepeatBuffer, ResidentLog, StreamAnalyzer
    from log_parser_amd.utils.synth import realistic_library
    dev = _dev(args)
    eng, _, trig = _engine(1000, dev, library=args.library)
    sets2, _ = realistic_library(1000, seed=99)
    eng2 = Engine(CompiledLibrary(sets2, ScoringParams()), eng.config, device=dev)
    big = eng if eng.lib.halo >= eng2.lib.halo else eng2
    block = make_log(200_000, trig, seed=6, hit_rate=0.004, aux_rate=0.01, stack_rate=0.01).encode()
    total = (args.gb << 30) // len(block) * len(block)
    src = RepeatBuffer(block, total)
    chunk = (args.chunk_mb << 20) if args.chunk_mb else None
    _sync(dev)
    t0 = time.perf_counter()
    res = ResidentLog.load(src, big, chunk_bytes=chunk)
    _sync(dev)
    load_s = time.perf_counter() - t0
    out = {"config": f"resident-{total / (1 << 30):.1f}GiB-reanalysis", "device": str(dev), "bytes": total,
           "chunks": len(res.chunks), "chunk_bytes": res.chunk_bytes, "load_s": round(load_s, 3),
           "load_GB_per_s": round(total / load_s / 1e9, 2), "analyses": []}
    for name, e in (("library-A", eng), ("library-B", eng2)):
        sa = StreamAnalyzer(e, chunk_bytes=res.chunk_bytes, topk=100, keep_events=False)
        sa.run(ResidentLog(res.chunks[:1], res.chunks[0][1], res.halo, res.chunk_bytes))    # warm (1 chunk)
        e.freq.reset_all()
        _sync(dev)
        t1 = time.perf_counter()
        r = sa.run(res)
        _sync(dev)
        dt = time.perf_counter() - t1
        out["analyses"].append({"library": name, "seconds": round(dt, 3), "lines": r.total_lines,
                                "lines_per_s": round(r.total_lines / dt, 1), "GB_per_s": round(total / dt / 1e9, 1),
                                "events": r.n_events, "highest": r.summary["highestSeverity"]})
    print(json.dumps(out))


def mode_concurrent(args):
    from log_parser_amd.serve.app import Batcher
    from log_parser_amd.utils.metrics import Metrics
    dev = _dev(args)
    eng, _, trig = _engine(1000, dev, library=args.library)
    rng = np.random.default_rng(0)
    sizes = rng.choice([20, 100, 500, 2000, 10000], size=args.requests, p=[0.3, 0.3, 0.2, 0.15, 0.05])
    pool = {s: [make_log(int(s), trig, seed=int(s) + k, hit_rate=0.01) for k in range(4)] for s in set(sizes.tolist())}
    reqs = [pool[int(s)][i % 4] for i, s in enumerate(sizes)]
    engines = [eng]
    ngpu = torch.cuda.device_count() if dev.type == "cuda" else 0
    for i in range(1, args.engines):     # one engine per GPU; several per GPU on a 1-GPU box
        d = torch.device("cuda", i % ngpu) if ngpu else dev
        engines.append(Engine(eng.lib, eng.config, device=d, freq=eng.freq))
    b = Batcher(engines, int(eng.config["engine.batch.max-requests"]), int(eng.config["engine.batch.max-bytes"]),
                float(eng.config["engine.batch.max-wait-ms"]), Metrics())
    for f in [b.submit(r) for r in reqs]:     # warm server: one untimed burst (staging buffers grown)
        f.result()
    lat = [0.0] * len(reqs)
    done = threading.Semaphore(0)

    def cb(i, t0):
        def _f(_fut):
            lat[i] = time.perf_counter() - t0
            done.release()
        return _f

    if args.timeline and b.pipe is not None:
        b.pipe.timeline = []
    t_start = time.perf_counter()
    for i, r in enumerate(reqs):              # all requests in flight at once (10k concurrent)
        t0 = time.perf_counter()
        b.submit(r).add_done_callback(cb(i, t0))
    for _ in reqs:
        done.acquire()
    wall = time.perf_counter() - t_start
    b.close()
    if args.timeline and b.pipe is not None:
        for st, n, a, z in b.pipe.timeline:
            print(f"{st:9s} n={n:5d} {1e3 * (a - t_start):8.2f} -> {1e3 * (z - t_start):8.2f} ms", file=sys.stderr)
    lat = np.array(lat)
    print(json.dumps({"config": f"concurrent-{args.requests}-requests-mixed", "device": str(dev), "engines": args.engines,
                      "p50_ms": round(float(np.median(lat)) * 1e3, 3), "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3),
                      "requests_per_s": round(len(reqs) / wall, 1), "lines_per_s": round(float(sizes.sum()) / wall, 1)}))


def mode_concurrent_http(args):
    """Config 5 as stated: N concurrent POST /parse requests over N keep-alive HTTP connections to
    the service process (native epoll front end -> continuous batcher -> GPU), mixed body sizes,
    realistic library. The native load generator (csrc/io/loadgen.cpp) opens every connection
    first, then sends one request on each at once; latency = first request byte -> last response
    byte. One untimed burst warms the server; the second is reported."""
    from log_parser_amd.native import N
    from log_parser_amd.serve.__main__ import raise_fd_limit
    from log_parser_amd.utils.numa import cgroup_throttling, cpu_budget, cpu_limits
    from log_parser_amd.utils.restbench import ServerProcess, collect_stages, stage_breakdown, write_library
    from log_parser_amd.utils.synth import realistic_library
    n = args.requests
    if raise_fd_limit() < n + 256:
        raise SystemExit(f"open-file limit too low for {n} connections")
    sets, trig = realistic_library(1000, seed=7)
    dev = "cpu" if args.device == "cpu" else ("cuda:0" if torch.cuda.is_available() else "cpu")
    if dev != "cpu":
        # the load generator on the GPU's socket, where the server binds itself (serve/__main__.py):
        # loopback traffic then stays on one socket (unbound, its threads landed on either socket of
        # the 256-CPU host and the burst rate halved in about half of the runs, profiles/r4_d)
        from log_parser_amd.utils.numa import bind_to_gpu_numa
        bind_to_gpu_numa(0)
    extra = [f"-Dengine.serve-devices={','.join([dev] * args.engines)}"] if args.engines > 1 else []
    if args.processes > 1:          # serving processes sharing one window (serve/procs.py)
        extra = [f"-Dserver.processes={args.processes}"]
    if args.timeline:
        extra.append("-Dserver.stage-timeline=true")
    srv = ServerProcess(write_library(sets), dev, http="native", extra=extra + list(args.server_opt or []),
                        log_path=args.server_log)
    conn_phases = None
    try:
        if not srv.wait_ready(workers=max(args.processes, 1)):
            raise SystemExit("server did not come up")
        rng = np.random.default_rng(0)
        sizes_set = [20, 100, 500, 2000, 10000]
        sizes = rng.choice(sizes_set, size=n, p=[0.3, 0.3, 0.2, 0.15, 0.05])
        msgs, lines_of = [], []
        for s_ in sizes_set:
            for k in range(4):
                body = json.dumps({"pod": {"metadata": {"name": f"pod-{s_}-{k}"}},
                                   "logs": make_log(int(s_), trig, seed=int(s_) + k, hit_rate=0.01)}).encode()
                msgs.append(b"POST /parse HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: application/json\r\n"
                            b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
                lines_of.append(int(s_))
        idx = np.array([sizes_set.index(int(s_)) * 4 + i % 4 for i, s_ in enumerate(sizes)], np.int32)
        N.http_burst("127.0.0.1", srv.port, msgs, idx[:min(n, 2000)], 300.0, args.client_threads)  # warm-up
        workers = max(args.processes, 1)
        st0 = collect_stages(srv.port, workers)
        thr0 = cgroup_throttling()
        ss0 = srv.sched_ns()
        cpu0, cli0 = srv.cpu_seconds(), time.process_time()
        sampler = None
        if args.sample_threads:      # every server thread's state / wait channel / syscall, every 1 ms
            from log_parser_amd.utils.threadsample import ThreadSampler
            sampler = ThreadSampler(srv._pids(), 0.001).start()
        lat, st, wall, done = N.http_burst("127.0.0.1", srv.port, msgs, idx, 600.0, args.client_threads)
        if sampler is not None:
            sampler.stop()
        cpu_srv, cpu_cli = srv.cpu_seconds() - cpu0, time.process_time() - cli0
        ss1 = srv.sched_ns()
        thr1 = cgroup_throttling()
        throttle = {k: round(thr1[k] - thr0[k], 3) for k in thr1} if thr0 and thr1 else {}
        # server thread-seconds on a CPU vs runnable-but-waiting for one during the burst (schedstat;
        # the load generator's threads exit with the burst, so only the server is counted)
        sched = {"server_run_s": round((ss1[0] - ss0[0]) / 1e9, 3), "server_wait_s": round((ss1[1] - ss0[1]) / 1e9, 3)}
        st1 = collect_stages(srv.port, workers)
        breakdown = stage_breakdown(st0, st1, wall)
        conn_phases = None
        if args.timeline:           # per /parse response of the burst: where its time went (native front end)
            recs = [r for d in st1.values() for r in d.get("conns", []) if r[5] >= 0]
            if recs:
                a = np.array(recs)
                a = a[a[:, 5] >= a[:, 5].max() - wall - 0.05]          # the timed burst's responses
                t0 = a[:, 2].min()

                def q(x):
                    return [round(float(np.percentile(x, k)) * 1e3, 3) for k in (50, 90, 99, 100)]
                conn_phases = {"responses": int(len(a)),
                               "ms_p50_p90_p99_max": {"first_byte_after_burst_start": q(a[:, 2] - t0),
                                                      "receive": q(a[:, 3] - a[:, 2]),
                                                      "parsed_to_handed_back": q(a[:, 4] - a[:, 3]),
                                                      "send": q(a[:, 5] - a[:, 4])},
                               "per_io_thread": {str(int(k)): int((a[:, 0] == k).sum()) for k in np.unique(a[:, 0])},
                               "parsed_by_ms": np.histogram(a[:, 3] - t0, bins=np.arange(0, wall * 1e3 + 1, 10) / 1e3)[0].tolist()}
            for pid, d in st1.items():
                t_end = d["now"]
                ev = [e for e in d.get("timeline", []) if e[3] >= t_end - wall - 0.05]
                t0 = min((e[2] for e in ev), default=t_end)
                for stg, nreq, a, z in ev:
                    print(f"pid {pid} {stg:9s} n={nreq:5d} {1e3 * (a - t0):8.2f} -> {1e3 * (z - t0):8.2f} ms",
                          file=sys.stderr)
    finally:
        srv.stop()
    ok = lat >= 0
    lines = float(np.array(lines_of)[idx].sum())
    print(json.dumps({"config": f"concurrent-http-{n}-connections-mixed-realistic", "device": dev,
                      "engines": args.engines, "processes": args.processes, "connections": n,
                      "client_threads": args.client_threads,
                      "completed": int(done),
                      "status_200": int((st == 200).sum()),
                      "p50_ms": round(float(np.median(lat[ok])) * 1e3, 3),
                      "p99_ms": round(float(np.percentile(lat[ok], 99)) * 1e3, 3),
                      "max_ms": round(float(lat[ok].max()) * 1e3, 3),
                      "requests_per_s": round(int(done) / wall, 1), "lines_per_s": round(lines / wall, 1),
                      "wall_s": round(wall, 3), "bytes": int(sum(len(msgs[i]) for i in idx)),
                      "breakdown": breakdown,
                      # CPUs busy during the burst (server processes / the load generator in this
                      # process): against the host's CPU budget, the measure of a host-bound burst
                      "cpus_busy": {"server": round(cpu_srv / wall, 2), "client": round(cpu_cli / wall, 2),
                                    "budget": cpu_budget(), **cpu_limits()},
                      # CFS quota throttling during the burst (cgroup cpu.stat deltas)
                      "cgroup_throttling": throttle,
                      "sched": sched,
                      "thread_states": sampler.summary() if sampler is not None else None,
                      "conn_phases": conn_phases,
                      "thread_samples": sampler.samples if sampler is not None else 0,
                      "transport": "native HTTP/1.1 front end, one keep-alive connection per request, 127.0.0.1"}))


def mode_golden(args):
    sets, trig = make_library(20, seed=3, n_sets=2)
    logs = make_log(args.lines, trig, seed=4, hit_rate=0.01)
    p = ScoringParams()
    t0 = time.perf_counter()
    r = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    dt = time.perf_counter() - t0
    print(json.dumps({"config": f"golden-python-proxy-{args.lines}-lines-20-patterns", "seconds": round(dt, 3),
                      "lines_per_s": round(r["metadata"]["totalLines"] / dt, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["rest", "rest_gpu", "single", "stream", "concurrent", "concurrent_http", "resident",
                                     "golden"])
    ap.add_argument("--gb", type=int, default=50, help="resident: GiB of log kept in HBM")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--lines", type=int, default=None)
    ap.add_argument("--patterns", type=int, default=4000)
    ap.add_argument("--steps", type=int, default=None, help="timed iterations (single: 20, else 5)")
    ap.add_argument("--requests", type=int, default=None)
    ap.add_argument("--chunk-mb", type=int, default=0, help="stream / resident chunk MiB (0 = from free HBM)")
    ap.add_argument("--timeline", action="store_true", help="concurrent: print the pipeline stage timeline")
    ap.add_argument("--sample-threads", action="store_true",
                    help="concurrent_http: sample every server thread's state / wait channel every 1 ms")
    ap.add_argument("--engines", type=int, default=1, help="concurrent: serving engines (one per GPU)")
    ap.add_argument("--processes", type=int, default=1,
                    help="concurrent_http: serving processes sharing one frequency window (server.processes)")
    ap.add_argument("--server-opt", action="append", help="concurrent_http: extra -Dkey=value for the server")
    ap.add_argument("--client-threads", type=int, default=8,
                    help="concurrent_http: load-generator threads (they share the host's CPUs with the server)")
    ap.add_argument("--server-log", default=None, help="concurrent_http: server stdout / stderr to this file")
    ap.add_argument("--http", default="native", choices=["native", "uvicorn"], help="rest: HTTP front end")
    ap.add_argument("--library", default="realistic", choices=["realistic", "synthetic"],
                    help="single / stream / concurrent: pattern library kind")
    args = ap.parse_args()
    defaults = {"rest": (10_000, 50), "rest_gpu": (10_000, 100), "single": (1_000_000, None), "stream": (1_000_000_000, None),
                "concurrent": (None, 10_000), "concurrent_http": (None, 10_000), "resident": (None, None),
                "golden": (10_000, None)}
    dl, dr = defaults[args.mode]
    args.lines = args.lines or dl
    args.requests = args.requests or dr
    args.steps = args.steps or (20 if args.mode == "single" else 5)
    globals()["mode_" + args.mode](args)


if __name__ == "__main__":
    main()
