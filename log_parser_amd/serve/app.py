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
import os
import sys
import threading
import time
from collections import deque
from concurrent.futures import Future
from typing import List, Optional

import torch
from fastapi import FastAPI, Request
from fastapi.responses import Response

from ..engine import Engine, ProcessWindowTurn, SharedWindowTurn
from ..frequency import MirroredFrequencyState
from ..models.compiled import CompiledLibrary
from ..models.library import load_pattern_directory
from ..native import N
from ..ops.kernels import padded_len as K_padded
from .pipeline import BatchPipeline
from ..utils.config import Config
from ..utils.metrics import Metrics

log = logging.getLogger("log_parser_amd.server")

INVALID = b'{"error":"Invalid PodFailureData provided"}'
UNSUPPORTED = b'{"error":"Content-Type must be application/json"}'


def json_media_type(content_type: Optional[str]) -> bool:
    """``@Consumes(MediaType.APPLICATION_JSON)`` (Parse.java:42): the media type of the request's
    Content-Type (parameters such as ``charset`` ignored, case-insensitive) must be
    application/json, else HTTP 415. A request without the header is accepted (JAX-RS leaves it to
    the implementation; parity unpinned -- no JVM here to check Quarkus)."""
    if content_type is None:
        return True
    return content_type.split(";", 1)[0].strip().lower() == "application/json"


class Batcher:
    """Continuous batcher. One worker thread per engine; each engine owns one GPU (or the CPU).

    With several engines (``engine.serve-devices``) batches are analysed concurrently on all
    GPUs of the node; every batch gets an arrival sequence number and reads / records the shared
    frequency state inside a ``FrequencyTurn`` in that order, so results are identical to serving
    the same batches one after another on one GPU."""

    def __init__(self, engines, max_requests: int, max_bytes: int, max_wait_ms: float, metrics: Metrics,
                 turn: Optional[SharedWindowTurn] = None):
        """``turn``: a ``ProcessWindowTurn`` when this process is one of several serving processes
        sharing one window (serve/procs.py): each batch then draws its arrival ticket from the
        shared segment when it enters the device stage."""
        self.engines: List[Engine] = list(engines) if isinstance(engines, (list, tuple)) else [engines]
        self.engine = self.engines[0]
        self.proc = isinstance(turn, ProcessWindowTurn)
        self.turn: Optional[SharedWindowTurn] = turn if turn is not None else (
            SharedWindowTurn() if len(self.engines) > 1 else None)
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
        si = float(self.engine.config.get("server.switch-interval-ms", 0.0) or 0.0)
        if si > 0:
            sys.setswitchinterval(si / 1000.0)
        # one engine: pack / device / emit of consecutive batches overlap (serve/pipeline.py)
        self.pipe: Optional[BatchPipeline] = (BatchPipeline(self.engine, self.device_stage, metrics.observe_batch)
                                              if len(self.engines) == 1 else None)
        pre = int(self.engine.config.get("engine.batch.prewarm-bytes", 0) or 0)
        for e in self.engines:      # pinned stages sized before the first request, not inside a burst
            if pre > 0 and e.device.type == "cuda":
                e._stage_pool.prewarm(K_padded(min(pre, max_bytes)), max(1, min(pre, max_bytes) // 40))
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
        if self.pipe is not None:
            self.pipe.close()

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
        from ..utils.threadsample import set_os_thread_name
        set_os_thread_name("lp-batcher")
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
            if self.pipe is not None and not (len(batch) == 1 and self.pipe.idle() and not self._q):
                # under load: hand the batch to the pipeline and form the next one meanwhile; a
                # lone request on an idle server runs inline (no thread hand-offs)
                self.pipe.submit([b[0] for b in batch], self._completion(batch))
                continue
            try:
                t0 = time.perf_counter()
                if self.pipe is not None:
                    outs = self.pipe.run_inline([b[0] for b in batch])      # observes the batch
                else:
                    outs = self.analyze(eng, [b[0] for b in batch], None if self.proc else seq)
                    self.metrics.observe_batch(len(batch), time.perf_counter() - t0)
                for (_, fut, _), o in zip(batch, outs):
                    fut.set_result(o)
            except Exception as e:  # noqa: BLE001 - propagate to every waiter
                log.exception("batch failed")
                for _, fut, _ in batch:
                    if not fut.done():
                        fut.set_exception(e)
            finally:
                if self.turn is not None and self.pipe is None:
                    self.turn.done(seq)    # no-op after a successful batch; unblocks later ones

    @staticmethod
    def _completion(batch):
        def done(outs, exc):
            if exc is not None:
                for _, fut, _ in batch:
                    if not fut.done():
                        fut.set_exception(exc)
                return
            for (_, fut, _), o in zip(batch, outs):
                fut.set_result(o)
        return done

    def device_stage(self, job, eng: Optional[Engine] = None, seq: int = 0) -> None:
        """Pipeline device stage with the same CPU fallback as ``analyze``. Several serving
        processes: the batch draws its arrival ticket itself, late (``seq`` None: the native runner
        once its matching is done, the Python paths right before their window section), and
        releases it on every exit."""
        eng = eng or self.engine
        if self.proc:
            seq = None
        try:
            eng.device_batch(job, self.turn, seq)
        except Exception:  # noqa: BLE001
            if not self.fallback_cpu:
                raise
            log.exception("device batch failed; serving it from the CPU backend")
            job.outs = self._cpu(eng).analyze_batch_json(job.logs, self.turn, seq, record=not job.recorded)

    def _cpu(self, eng: Engine) -> Engine:
        """The CPU backend for one failed batch. A device-resident window is not touched by it
        directly (the device may be the thing that failed): the fallback reads a host copy of the
        window (empty when the device cannot be read) and its record goes to that copy and, best
        effort, back to the device window."""
        with self._cpu_lock:
            self.metrics.device_failures += 1
            freq = eng.freq
            if getattr(freq, "device_resident", False):
                freq = MirroredFrequencyState(freq)
            elif self._cpu_engine is not None:
                return self._cpu_engine
            cpu = Engine(eng.lib, eng.config, device=torch.device("cpu"), freq=freq)
            cpu.fault_every = cpu.fault_after_record = 0
            if not getattr(eng.freq, "device_resident", False):
                self._cpu_engine = cpu
            return cpu

    def analyze(self, eng: Engine, logs: List[str], seq: Optional[int]) -> List[bytes]:
        """GPU batch; on a device failure (HIP error, OOM, lost device) serve the batch from the CPU
        backend — same library tables, a host copy of the frequency window — for availability only
        (SURVEY §5.3), and report it in /metrics. A batch whose counts already entered the window
        (failure after the record) is not recorded again."""
        job = eng.pack_batch(logs)
        try:
            try:
                eng.device_batch(job, self.turn, seq)
                return eng.emit_batch(job)
            finally:
                eng.release_batch(job)
        except Exception:  # noqa: BLE001
            if not self.fallback_cpu:
                raise
            log.exception("device batch failed; serving it from the CPU backend")
            return self._cpu(eng).analyze_batch_json(logs, self.turn, seq, record=not job.recorded)


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


class Service:
    """The service logic shared by both HTTP front ends (FastAPI/uvicorn and the native epoll
    server, ``serve/native_http.py``): library + engines + batcher + metrics, the /parse flow and
    the health / metrics / admin routes (reference surface: Parse.java; additions SURVEY §5.3-5.5)."""

    JSON = "application/json"

    def __init__(self, config: Optional[Config] = None, engine: Optional[Engine] = None, proc=None):
        """``proc``: this process's ``serve.procs.WorkerContext`` when it is one of several serving
        processes (one engine here, the frequency window shared with the others)."""
        self.config = config or Config.load()
        self.metrics = Metrics()
        self._engine = engine
        self._batcher: Optional[Batcher] = None
        self._lock = threading.Lock()
        self.proc = proc

    # ---- lifecycle
    def engine(self) -> Engine:
        with self._lock:
            if self._engine is None:
                cfg = self.config
                sets = load_pattern_directory(cfg["pattern.directory"])
                lib = CompiledLibrary(sets, cfg.scoring, max_dfa_states=int(cfg["engine.dfa-max-states"]),
                                  nfa_engine=str(cfg["engine.nfa-engine"]))
                log.info("compiled library: %s", lib.summary())
                if self.proc is not None:      # one of several serving processes: the shared window
                    self._engine = Engine(lib, cfg, freq=self.proc.frequency_state(lib, cfg))
                    snap = cfg["engine.frequency.snapshot-path"] if self.proc.owner else ""
                else:
                    self._engine = Engine(lib, cfg)
                    snap = cfg["engine.frequency.snapshot-path"]
                if snap:                       # resume the sliding window of a previous run
                    self._engine.freq.restore(snap)
                if self.proc is not None:
                    self.proc.window_ready()
            return self._engine

    def batcher(self) -> Batcher:
        eng = self.engine()
        with self._lock:
            if self._batcher is None:
                cfg = self.config
                if self.proc is not None:
                    self._batcher = Batcher([eng], int(cfg["engine.batch.max-requests"]),
                                            int(cfg["engine.batch.max-bytes"]), float(cfg["engine.batch.max-wait-ms"]),
                                            self.metrics, turn=ProcessWindowTurn(self.proc.shared))
                    return self._batcher
                engines = [eng]
                devs = serve_devices(cfg)
                if devs and devs[0] == eng.device:
                    devs = devs[1:]
                elif eng.device in devs:
                    devs.remove(eng.device)
                if getattr(eng.freq, "device_resident", False) and not self._device_window_ok(eng, devs):
                    # engines on other physical GPUs without a verified peer window: ONE host
                    # window shared by every engine (the pre-peer behaviour), seeded from the device
                    log.warning("serving on several GPUs with a shared host frequency window")
                    eng.freq = eng.freq.to_host_state()
                for dev in devs:                   # data-parallel serving: one engine per GPU (or stream)
                    engines.append(Engine(engines[0].lib, cfg, device=dev, freq=engines[0].freq))
                if len(engines) > 1:
                    log.info("serving on %d engines: %s", len(engines), [str(e.device) for e in engines])
                self._batcher = Batcher(engines, int(cfg["engine.batch.max-requests"]),
                                        int(cfg["engine.batch.max-bytes"]), float(cfg["engine.batch.max-wait-ms"]),
                                        self.metrics)
            return self._batcher

    def _device_window_ok(self, eng: Engine, devs: List[torch.device]) -> bool:
        """Whether the engines on ``devs`` can share the first engine's HBM window. Streams of the
        same GPU always can; other GPUs only with ``engine.serve.peer-window`` (the cross-GPU peer
        path is opt-in until a multi-GPU run has pinned it) and working peer access."""
        home = eng.freq.device.index or 0
        for dev in devs:
            if dev.type != "cuda":
                return False
            idx = dev.index if dev.index is not None else 0
            if idx == home:
                continue
            if not bool(self.config.get("engine.serve.peer-window", False)):
                return False
            if not N.enable_peer_access(idx, home):
                log.warning("no peer access from %s to %s for the shared window", dev, eng.freq.device)
                return False
        return True

    def close(self):
        if self._batcher is not None:
            self._batcher.close()
        path = self.config["engine.frequency.snapshot-path"]
        if path and self._engine is not None and (self.proc is None or self.proc.owner):
            self._engine.freq.snapshot(path)

    # ---- POST /parse (Parse.java:41-61)
    def submit_parse(self, logs, name: str, t0: float) -> Future:
        """A decoded request: INFO log, batch submission, metrics on completion."""
        log.info("Received analysis request for pod: %s", name or "<unknown>")
        fut = self.batcher().submit(logs)
        n = len(logs)

        def _done(f):
            if f.exception() is None:
                self.metrics.observe_request(200, time.perf_counter() - t0, n)
                log.info("Analysis complete for pod: %s.", name or "<unknown>")
        fut.add_done_callback(_done)
        return fut

    def decode_body(self, body: bytes, t0: float):
        """Raw /parse body -> (logs, pod name) or an immediate (status, content type, bytes) error.
        Decoded natively (csrc/io/json_in.cpp); unusual bodies (non-UTF-8 encodings, NaN literals,
        surrogate escapes) go through json.loads."""
        if len(body) > int(self.config["server.max-body-bytes"]):
            return 413, self.JSON, b'{"error":"request body too large"}'
        st, pod_ok, name, logs_kind, logs = N.parse_pod_request(body) if body else (1, False, None, 0, None)
        if st == 3:
            import json
            try:
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
            self.metrics.observe_request(400, time.perf_counter() - t0, 0)
            return 400, self.JSON, INVALID
        if logs_kind != 1:
            self.metrics.observe_request(400, time.perf_counter() - t0, 0)
            return 400, self.JSON, b'{"error":"PodFailureData.logs must be a string"}'
        return logs, name

    def parse_body(self, body: bytes, t0: float, content_type: Optional[str] = None):
        """Raw /parse body -> (status, content type, bytes) or a Future of the JSON bytes."""
        if not json_media_type(content_type):
            self.metrics.observe_request(415, time.perf_counter() - t0, 0)
            return 415, self.JSON, UNSUPPORTED
        r = self.decode_body(body, t0)
        if len(r) == 3:
            return r
        return self.submit_parse(r[0], r[1], t0)

    # ---- other routes
    def route(self, method: str, path: str, body: bytes = b""):
        import json
        path = path.split("?", 1)[0]
        j = lambda obj, code=200: (code, self.JSON, json.dumps(obj, separators=(",", ":")).encode())  # noqa: E731
        if path == "/health" and method == "GET":
            return j({"status": "UP"})
        if path == "/ready" and method == "GET":
            e = self._engine
            if e is None:
                return j({"status": "DOWN", "reason": "library not loaded"}, 503)
            w = {"index": self.proc.index if self.proc is not None else 0, "pid": os.getpid(),
                 "processes": self.proc.nproc if self.proc is not None else 1}
            return j({"status": "UP", "device": str(e.device), "library": e.lib.summary(), "worker": w,
                      "nativeRunner": e._runner not in (None, False)})
        if path == "/metrics" and method == "GET":
            if self._engine is not None:
                self.metrics.set_frequency(self._engine.freq.statistics())
                bt = self._engine.lib.host_bt
                self.metrics.bt_exhausted = int(bt.exhausted) if bt is not None else 0
            return 200, "text/plain; version=0.0.4", self.metrics.render().encode()
        if path == "/admin/config" and method == "GET":
            return j(dict(self.config.values))
        if path == "/admin/frequency":
            if method == "GET":
                return j(self.engine().freq.statistics())
            if method == "DELETE":
                self.engine().freq.reset_all()
                return j({"reset": "all"})
        if path.startswith("/admin/frequency/"):
            from urllib.parse import unquote
            pid = unquote(path[len("/admin/frequency/"):])
            if method == "GET":
                r = self.engine().freq.get_pattern_frequency(pid)
                return j(r) if r is not None else j({"error": "unknown pattern id"}, 404)
            if method == "DELETE":
                self.engine().freq.reset(pid)
                return j({"reset": pid})
        return j({"error": "not found"}, 404)


def create_app(config: Optional[Config] = None, engine: Optional[Engine] = None,
               service: Optional[Service] = None) -> FastAPI:
    """FastAPI front end (uvicorn) over ``Service``; ``server.http=native`` uses the epoll server."""
    svc = service or Service(config, engine)
    app = FastAPI(title="log_parser_amd", version="0.1.0")
    app.state.service = svc

    @app.on_event("startup")
    def _startup():
        svc.batcher()

    @app.on_event("shutdown")
    def _shutdown():
        svc.close()

    def _resp(r):
        code, ctype, data = r
        return Response(data, status_code=code, media_type=ctype)

    @app.post("/parse")
    async def parse(request: Request):
        t0 = time.perf_counter()
        r = svc.parse_body(await request.body(), t0, request.headers.get("content-type"))
        if isinstance(r, tuple):
            return _resp(r)
        return Response(await asyncio.wrap_future(r), media_type="application/json")

    @app.api_route("/{path:path}", methods=["GET", "DELETE"])
    def other(path: str, request: Request):
        return _resp(svc.route(request.method, "/" + path))

    return app
