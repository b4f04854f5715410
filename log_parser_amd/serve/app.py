"""REST service: ``POST /parse`` (reference ``Parse.java:23-62``) plus health, metrics and admin.

Behaviour kept from the reference:
* ``POST /parse`` consumes/produces ``application/json`` (``Parse.java:41-44``);
* body or ``pod`` null -> HTTP 400 ``{"error":"Invalid PodFailureData provided"}`` (``:45-49``);
* otherwise 200 + ``AnalysisResult`` (``:60``); INFO log per request (``:51,55-58``).

Additions: ``/health``, ``/ready``, Prometheus ``/metrics``,
``/admin/frequency`` statistics/reset (the reference has the service methods but no endpoint),
and a **continuous batcher**: requests that queue while a batch runs on the GPU are packed into
the next device batch (``Engine.analyze_batch_json``), so 10k concurrent small requests cost a few
large kernel launches instead of 10k small ones, while a request reaching an idle server starts
at once (``engine.batch.max-wait-ms`` > 0 additionally holds a batch open that long).

Deliberate differences: ``logs`` null -> 400 (the reference NPEs into a 500); a pod without
``metadata`` is accepted (logged as ``<unknown>``); per-match logging is DEBUG, not INFO.
"""
from __future__ import annotations

import asyncio
import gc
import logging
import threading
import time
from collections import deque
from concurrent.futures import Future
from typing import List, Optional

import torch
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, Response

from ..engine import Engine, FrequencyTurn
from ..models.compiled import CompiledLibrary
from ..models.library import load_pattern_directory
from ..native import N
from ..utils.config import Config
from ..utils.metrics import Metrics

log = logging.getLogger("log_parser_amd.server")

INVALID = b'{"error":"Invalid PodFailureData provided"}'


class Batcher:
    """Continuous batcher. One worker thread per engine; each engine owns one GPU (or the CPU).

    With several engines (``engine.serve-devices``) batches are analysed concurrently on all
    GPUs of the node; every batch gets an arrival sequence number and reads / records the shared
    frequency state inside a ``FrequencyTurn`` in that order, so results are identical to serving
    the same batches one after another on one GPU."""

    def __init__(self, engines, max_requests: int, max_bytes: int, max_wait_ms: float, metrics: Metrics):
        self.engines: List[Engine] = list(engines) if isinstance(engines, (list, tuple)) else [engines]
        self.engine = self.engines[0]
        self.turn: Optional[FrequencyTurn] = FrequencyTurn() if len(self.engines) > 1 else None
        self.max_requests = max_requests
        self.max_bytes = max_bytes
        self.max_wait = max_wait_ms / 1000.0
        self.metrics = metrics
        self.fallback_cpu = bool(self.engine.config.get("engine.fallback-cpu", True))
        self._cpu_engine: Optional[Engine] = None
        self._cpu_lock = threading.Lock()
        self._q: "deque[tuple]" = deque()
        self._cv = threading.Condition()
        self._stop = False
        self._seq = 0
        if bool(self.engine.config.get("server.gc-tuning", True)):
            # Every in-flight request holds a Future (+ Condition + RLock); with thousands in flight
            # the cyclic GC's full passes over the (torch-heavy) heap dominate submit cost
            # (12 us -> 2.6 us per request). Freeze the startup heap, collect young objects lazily.
            gc.collect()
            gc.freeze()
            gc.set_threshold(50_000, 50, 100)
        self._threads = [threading.Thread(target=self._loop, args=(e,), name=f"lp-batcher-{i}", daemon=True)
                         for i, e in enumerate(self.engines)]
        for t in self._threads:
            t.start()

    def submit(self, logs) -> Future:
        fut: Future = Future()
        with self._cv:
            self._q.append((logs, fut, time.perf_counter()))
            # wake a worker only when it can act: first request of a batch, or a full batch.
            # Notifying on every submit makes the worker threads contend for the GIL 10k times.
            n = len(self._q)
            if n == 1 or n == self.max_requests:
                self._cv.notify()
        return fut

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join(timeout=5)

    def _take(self):
        with self._cv:
            while not self._q and not self._stop:
                self._cv.wait()
            if self._stop and not self._q:
                return 0, []
            deadline = self._q[0][2] + self.max_wait
            while len(self._q) < self.max_requests and time.perf_counter() < deadline:
                self._cv.wait(timeout=max(0.0, deadline - time.perf_counter()))
            batch, size = [], 0
            while self._q and len(batch) < self.max_requests:
                item = self._q[0]
                if batch and size + len(item[0]) > self.max_bytes:
                    break
                batch.append(self._q.popleft())
                size += len(item[0])
            seq = self._seq
            self._seq += 1
            if self._q:
                self._cv.notify()          # more queued: let another (idle) worker take it
            return seq, batch

    def _loop(self, eng: Engine):
        if eng.device.type == "cuda":
            torch.cuda.set_device(eng.device)
            if len(self.engines) > 1:      # own stream per worker: engines sharing a GPU overlap
                torch.cuda.set_stream(torch.cuda.Stream(eng.device))
        while True:
            seq, batch = self._take()
            if not batch:
                if self._stop:
                    return
                continue
            try:
                t0 = time.perf_counter()
                outs = self._analyze(eng, [b[0] for b in batch], seq)
                self.metrics.observe_batch(len(batch), time.perf_counter() - t0)
                for (_, fut, _), o in zip(batch, outs):
                    fut.set_result(o)
            except Exception as e:  # noqa: BLE001 - propagate to every waiter
                log.exception("batch failed")
                for _, fut, _ in batch:
                    if not fut.done():
                        fut.set_exception(e)
            finally:
                if self.turn is not None:
                    self.turn.done(seq)    # no-op after a successful batch; unblocks later ones

    def _analyze(self, eng: Engine, logs: List[str], seq: int) -> List[bytes]:
        """GPU batch; on a device failure (HIP error, OOM, lost device) serve the batch from the CPU
        backend — same library tables and the same frequency state — for availability only
        (SURVEY §5.3), and report it in /metrics."""
        try:
            return eng.analyze_batch_json(logs, self.turn, seq)
        except Exception:  # noqa: BLE001
            if not self.fallback_cpu:
                raise
            log.exception("device batch failed; serving it from the CPU backend")
            with self._cpu_lock:
                self.metrics.device_failures += 1
                if self._cpu_engine is None:
                    self._cpu_engine = Engine(eng.lib, eng.config, device=torch.device("cpu"), freq=eng.freq)
                    self._cpu_engine.fault_every = 0
                return self._cpu_engine.analyze_batch_json(logs, self.turn, seq)


def serve_devices(config: Config) -> List[torch.device]:
    """``engine.serve-devices``: "" = the single ``engine.device``; "all" = every visible GPU;
    or a comma list ("cuda:0,cuda:1")."""
    spec = str(config.get("engine.serve-devices", "") or "").strip()
    if not spec:
        return []
    if spec == "all":
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        return [torch.device("cuda", i) for i in range(n)] or [torch.device("cpu")]
    return [torch.device(x.strip()) for x in spec.split(",") if x.strip()]


def create_app(config: Optional[Config] = None, engine: Optional[Engine] = None) -> FastAPI:
    config = config or Config.load()
    app = FastAPI(title="log_parser_amd", version="0.1.0")
    metrics = Metrics()
    state = {"engine": engine, "batcher": None}

    def _engine() -> Engine:
        if state["engine"] is None:
            sets = load_pattern_directory(config["pattern.directory"])
            lib = CompiledLibrary(sets, config.scoring, max_dfa_states=int(config["engine.dfa-max-states"]))
            log.info("compiled library: %s", lib.summary())
            state["engine"] = Engine(lib, config)
        return state["engine"]

    def _batcher() -> Batcher:
        if state["batcher"] is None:
            engines = [_engine()]
            for dev in serve_devices(config):     # data-parallel serving: one engine per GPU
                if dev != engines[0].device:
                    engines.append(Engine(engines[0].lib, config, device=dev, freq=engines[0].freq))
            if len(engines) > 1:
                log.info("serving on %d engines: %s", len(engines), [str(e.device) for e in engines])
            state["batcher"] = Batcher(engines, int(config["engine.batch.max-requests"]),
                                       int(config["engine.batch.max-bytes"]), float(config["engine.batch.max-wait-ms"]),
                                       metrics)
        return state["batcher"]

    @app.on_event("startup")
    def _startup():
        _batcher()

    @app.on_event("shutdown")
    def _shutdown():
        if state["batcher"] is not None:
            state["batcher"].close()
        path = config["engine.frequency.snapshot-path"]
        if path and state["engine"] is not None:
            state["engine"].freq.snapshot(path)

    @app.post("/parse")
    async def parse(request: Request):
        t0 = time.perf_counter()
        body = await request.body()
        if len(body) > int(config["server.max-body-bytes"]):
            return JSONResponse({"error": "request body too large"}, status_code=413)
        # native single-pass decode (csrc/io/json_in.cpp): validates the JSON and returns the
        # `logs` string as UTF-8 bytes without building the object tree; unusual bodies
        # (non-UTF-8 encodings, NaN literals, surrogate escapes) go through json.loads
        st, pod_ok, name, logs_kind, logs = N.parse_pod_request(body) if body else (1, False, None, 0, None)
        if st == 3:
            try:
                import json
                data = json.loads(body)
            except ValueError:
                data = None
            st = 0 if isinstance(data, dict) else 1
            if st == 0:
                pod_ok = data.get("pod") is not None
                logs = data.get("logs")
                logs_kind = 1 if isinstance(logs, str) else (0 if logs is None else 2)
                pod = data["pod"] if isinstance(data.get("pod"), dict) else {}
                md = pod.get("metadata")
                name = md.get("name") if isinstance(md, dict) else None
                name = name if isinstance(name, str) else None
        if st != 0 or not pod_ok:
            metrics.observe_request(400, time.perf_counter() - t0, 0)
            return Response(INVALID, status_code=400, media_type="application/json")
        if logs_kind != 1:
            metrics.observe_request(400, time.perf_counter() - t0, 0)
            return JSONResponse({"error": "PodFailureData.logs must be a string"}, status_code=400)
        name = name or "<unknown>"
        log.info("Received analysis request for pod: %s", name)
        fut = _batcher().submit(logs)
        out = await asyncio.wrap_future(fut)
        metrics.observe_request(200, time.perf_counter() - t0, len(logs))
        log.info("Analysis complete for pod: %s.", name)
        return Response(out, media_type="application/json")

    @app.get("/health")
    def health():
        return {"status": "UP"}

    @app.get("/ready")
    def ready():
        e = state["engine"]
        if e is None:
            return JSONResponse({"status": "DOWN", "reason": "library not loaded"}, status_code=503)
        return {"status": "UP", "device": str(e.device), "library": e.lib.summary()}

    @app.get("/metrics")
    def prom():
        e = state["engine"]
        if e is not None:
            metrics.set_frequency(e.freq.statistics())
        return PlainTextResponse(metrics.render(), media_type="text/plain; version=0.0.4")

    @app.get("/admin/frequency")
    def freq_stats():
        return _engine().freq.statistics()

    @app.get("/admin/frequency/{pid}")
    def freq_one(pid: str):
        r = _engine().freq.get_pattern_frequency(pid)
        if r is None:
            return JSONResponse({"error": "unknown pattern id"}, status_code=404)
        return r

    @app.delete("/admin/frequency/{pid}")
    def freq_reset(pid: str):
        _engine().freq.reset(pid)
        return {"reset": pid}

    @app.delete("/admin/frequency")
    def freq_reset_all():
        _engine().freq.reset_all()
        return {"reset": "all"}

    @app.get("/admin/config")
    def cfg():
        return dict(config.values)

    return app
