"""Native HTTP/1.1 front end of the REST service (``server.http=native``, the default).

The C++ epoll server (``csrc/io/http_server.cpp``) owns the sockets: it parses requests, answers
``GET /health`` and malformed ``/parse`` bodies itself (HTTP 400, ``Parse.java:45-49``), and validates
``POST /parse`` bodies (``csrc/io/json_in.cpp``). One Python pump thread drains the requests in bulk
with the GIL released and hands them to the continuous batcher; with one engine (direct mode) the
log strings stay JSON-escaped in their receive buffers (``N.RawLogs``) until the engine's packer
unescapes them straight into its pinned stage, otherwise they are unescaped to UTF-8 bytes while
draining. Responses go back through ``HttpServer.respond`` from the batcher's completion callbacks.
Every other route (``/ready``, ``/metrics``, ``/admin/*``, the json.loads fallback of exotic
``/parse`` bodies) is served by the same ``Service`` methods as the FastAPI front end.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time
from typing import Optional

from ..native import N
from ..utils.batchlog import log_lines
from .app import Service

log = logging.getLogger("log_parser_amd.server")


class NativeHttpFrontend:
    def __init__(self, service: Service, host: str = "0.0.0.0", port: int = 8080, io_threads: int = 2):
        self.svc = service
        b = self.svc.batcher()                           # compile the library before accepting
        if b.pipe is not None and bool(service.config.get("server.stage-timeline", False)):
            b.pipe.timeline = []
        cfg = service.config
        trace = bool(cfg.get("server.trace-requests", False))
        restore = self._l3_affinity(cfg, io_threads, b)
        try:
            self._start(cfg, host, port, io_threads, trace)
            if restore is not None:
                # IO threads leave the L3 group under a burst of connections (config 5: ~80k vs 63-69k
                # req/s squeezed onto one CCD, profiles/r6_g) and come back when few remain
                self.srv.set_affinity_sets(sorted(os.sched_getaffinity(0)), sorted(restore), 64, 8)
        finally:
            if restore is not None:
                os.sched_setaffinity(0, restore)
        log.info("native HTTP front end on %s:%d (%d IO threads)", host, self.port, io_threads)

    @staticmethod
    def _l3_affinity(cfg, io_threads: int, b):
        """``server.l3-affinity``: this (creating) thread moves onto the CPUs of one last-level cache
        while the IO threads and the pump start -- they inherit it -- and returns the set to restore.
        Only with a GPU engine in direct mode and an L3 group that holds them all."""
        if not bool(cfg.get("server.l3-affinity", True)) or b.pipe is None or not hasattr(os, "sched_getaffinity"):
            return None
        eng = b.pipe.engine
        if eng.device.type != "cuda":
            return None
        from ..utils.numa import l3_groups, one_per_core
        allowed = os.sched_getaffinity(0)
        groups = l3_groups(allowed)
        if len(groups) < 2 or len(groups[0]) < io_threads + 2:
            return None
        # one hardware thread per core when that leaves a core for each IO thread, the pump and the
        # decode helper (a body's receiving IO thread and the helper decoding it share a core's units
        # on SMT siblings); else the whole L3 group: a burst of many connections needs every IO thread
        # (config 5 on 8 single-thread cores: 66-69k req/s against 80k unpinned, profiles/r6_g)
        cpus = one_per_core(groups[0])
        if len(cpus) < io_threads + 3:
            cpus = groups[0]
        os.sched_setaffinity(0, cpus)
        log.info("IO threads and pump on %d CPUs (one per core) of one L3: %s", len(cpus), sorted(cpus))
        return allowed

    def _start(self, cfg, host: str, port: int, io_threads: int, trace: bool) -> None:
        b = self.svc.batcher()
        self.srv = N.HttpServer(host, port, io_threads, int(cfg["server.max-body-bytes"]),
                                float(cfg["server.idle-timeout-s"]), io_spin_us=float(cfg["server.io-spin-us"]),
                                pump_spin_us=float(cfg["server.pump-spin-us"]),
                                quickack=bool(cfg["server.tcp-quickack"]), rcvbuf=int(cfg["server.rcvbuf-bytes"]),
                                trace=trace, conn_trace=bool(cfg.get("server.stage-timeline", False)),
                                prefetch=bool(cfg["server.prefetch-logs"]),
                                io_decode_max_conns=int(cfg["server.io-decode-max-conns"]))
        self.port = self.srv.port
        eng = b.pipe.engine if b.pipe is not None else None
        npin = int(cfg["server.pinned-decode-buffers"])
        if npin > 0 and eng is not None and eng.device.type == "cuda":
            # bodies >= 256 KiB are decoded by the IO threads into pinned buffers that the engine stages
            # in place (Engine._stage_docs): up to `npin` such buffers, then pageable ones
            self.srv.set_pinned_decode(npin, 256 << 10)
        self._stop = threading.Event()
        # server.trace-requests: per /parse request on stderr -- receive / validate (native side),
        # queue (body complete -> drained by the pump) and engine (drained -> response queued)
        # microseconds (tools/parse_tail.py)
        self._trace = {} if trace else None
        # pump thread's busy time: turning drained requests into a batch (dispatch) and, for an
        # inline batch, its responses (complete)
        self._pump_s = {"dispatch": 0.0, "complete_inline": 0.0}
        self._t = threading.Thread(target=self._pump, name="lp-http-pump", daemon=True)
        self._t.start()

    def _reply(self, rid: int, r) -> None:
        code, ctype, data = r
        self.srv.respond(rid, code, ctype, data)

    def _on_done(self, rid: int):
        def cb(fut):
            try:
                self.srv.respond(rid, 200, "application/json", fut.result())
            except Exception as e:  # noqa: BLE001 - the batch failed: 500 to this client
                log.error("request failed: %s", e)
                self.srv.respond(rid, 500, "application/json", b'{"error":"internal error"}')
        return cb

    def _pump(self) -> None:
        from ..utils.threadsample import set_os_thread_name
        set_os_thread_name("lp-pump")
        b = self.svc.batcher()
        direct = b.pipe is not None
        while not self._stop.is_set():
            # direct mode: /parse logs stay JSON-escaped in their receive buffers (N.RawLogs) and
            # are unescaped by the engine's packer straight into its pinned stage
            reqs = self.srv.next_requests(b.max_requests, 100, direct)
            if not reqs:
                continue
            td = time.perf_counter()
            batch = []
            for req in reqs:
                rid, kind = req[0], req[1]
                t0 = time.perf_counter()
                try:
                    if kind == 0:                            # validated POST /parse
                        _, _, logs, name, t_arr = req
                        if self._trace is not None:
                            self._trace[rid] = t_arr
                        if direct:          # "Received ..." is logged with the response (off the clock)
                            batch.append((rid, logs, name, t0))
                        else:
                            self.svc.submit_parse(logs, name, t0).add_done_callback(self._on_done(rid))
                        continue
                    _, _, method, path, body, _ = req
                    if path.split("?", 1)[0] == "/parse":
                        if method != "POST":
                            self._reply(rid, (405, "application/json", b'{"error":"method not allowed"}'))
                            continue
                        r = self.svc.decode_body(body, t0)       # json.loads fallback bodies
                        if len(r) == 3:
                            self._reply(rid, r)
                        elif direct:        # the engine is owned by this thread: same batch path
                            batch.append((rid, r[0], r[1], t0))
                        else:
                            self.svc.submit_parse(r[0], r[1], t0).add_done_callback(self._on_done(rid))
                        continue
                    if path == "/admin/stages" and method == "GET":
                        self._reply(rid, (200, "application/json", json.dumps(self.stages()).encode()))
                        continue
                    self._reply(rid, self.svc.route(method, path, body))
                except Exception as e:  # noqa: BLE001
                    log.exception("request handling failed")
                    self._reply(rid, (500, "application/json", ('{"error":"%s"}' % type(e).__name__).encode()))
            if batch:
                self._pump_s["dispatch"] += time.perf_counter() - td
                if b.pipe is not None and b.pipe.timeline is not None:
                    b.pipe.timeline.append(("drain", len(batch), td, time.perf_counter()))
                self._run_direct(b, batch)

    def _run_direct(self, b, batch) -> None:
        """Single engine: the pump thread is the continuous batcher -- everything that queued while
        the previous batch ran forms the next batch, with no hand-off to the batcher's worker (which
        never sees a request in this mode: every /parse, including the json.loads-fallback bodies,
        comes through here). A lone request on an idle pipeline runs inline on this thread (lowest
        latency); under load, batches go through the pack / device / emit pipeline."""
        logs = [x[1] for x in batch]
        if len(batch) == 1 and b.pipe.idle() and self.srv.pending() == 0:
            try:
                outs = b.pipe.run_inline(logs)
            except Exception as e:  # noqa: BLE001
                log.exception("batch failed")
                self._batch_done(batch, None, e)
                return
            t = time.perf_counter()
            self._batch_done(batch, outs, None)
            self._pump_s["complete_inline"] += time.perf_counter() - t
        else:
            b.pipe.submit(logs, lambda outs, exc: self._batch_done(batch, outs, exc))

    def _batch_done(self, batch, outs, exc) -> None:
        """Responses first (one native call for the batch), then the reference's per-request INFO
        lines (Parse.java:51,55-58: received, complete) written for the whole batch at once
        (utils/batchlog.py: a logging record per line cost 32 us of GIL time per request)."""
        names = [x[2] or "<unknown>" for x in batch]
        if exc is not None:
            err = ('{"error":"%s"}' % type(exc).__name__).encode()
            self.srv.respond_many([x[0] for x in batch], 500, "application/json", [err] * len(batch))
            log_lines(log, logging.INFO, ["Received analysis request for pod: " + n for n in names])
            return
        self.srv.respond_many([x[0] for x in batch], 200, "application/json", list(outs))
        now = time.perf_counter()
        if self._trace is not None:
            for rid, _, _, ta in batch:
                if rid in self._trace:
                    sys.stderr.write("lp-parse-trace queue_us %.1f engine_us %.1f\n" % (
                        (ta - self._trace.pop(rid)) * 1e6, (now - ta) * 1e6))
        self.svc.metrics.observe_requests(200, [now - x[3] for x in batch], sum(len(x[1]) for x in batch))
        lines = []
        for n in names:
            lines.append("Received analysis request for pod: " + n)
            lines.append("Analysis complete for pod: " + n + ".")
        log_lines(log, logging.INFO, lines)

    def stages(self) -> dict:
        """Per-stage busy seconds of this process (GET /admin/stages): the native side's receive /
        validate / queue / handoff / send sums (HttpServer.stage_stats) and the pump + pipeline
        threads' dispatch / pack / device / emit / complete sums, with request and batch counts."""
        out = {"pid": os.getpid(), "native": self.srv.stage_stats(), "pump": dict(self._pump_s)}
        pipe = self.svc.batcher().pipe
        if pipe is not None:
            out["pipeline"] = dict(pipe.stage_s)
            out["batches"] = pipe.batches
            out["requests"] = pipe.requests
            if pipe.timeline is not None:
                out["timeline"] = list(pipe.timeline)
                # per /parse response since the last call: (IO thread, accept, first byte, parsed,
                # handed back, sent) -- perf_counter seconds
                out["conns"] = self.srv.conn_trace().tolist()
        out["now"] = time.perf_counter()
        return out

    def close(self) -> None:
        self._stop.set()
        self._t.join(timeout=5)
        self.srv.stop()
        self.svc.close()

    def serve_forever(self, stop: Optional[threading.Event] = None) -> None:
        try:
            while not (stop or self._stop).wait(1.0):
                pass
        except KeyboardInterrupt:
            pass
        finally:
            self.close()
