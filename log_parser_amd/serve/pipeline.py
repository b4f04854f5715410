"""Three-stage serving pipeline over consecutive batches of one engine.

A continuous batch spends its time in three places: packing the request bodies into pinned
staging memory + line index (host, ``Engine.pack_batch``), the device (H2D, match + score kernels,
one D2H and the frequency commit, ``Engine.device_batch``) and JSON emission (host,
``Engine.emit_batch``). Run back to back, a 2048-request batch costs the SUM of the three; here
they run on different threads for consecutive batches (pack of batch i+2 || device of i+1 ||
emission of i), so a burst is served at the rate of the slowest stage. The device stage is one
thread, so frequency state is still read and recorded in batch (= arrival) order -- results are
identical to serving the batches one after another. The engine's ``StagePool`` (3 pinned buffers)
bounds the batches in flight and back-pressures the producer.

Reference: the reference serves each request on a Quarkus worker thread, sequentially inside
(AnalysisService.java:50-122); batching and pipelining are additions (SURVEY §2.3 N-BATCH).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from typing import Callable, List, Optional, Sequence

import torch

from ..engine import Engine

log = logging.getLogger("log_parser_amd.server")

Done = Callable[[Optional[List[bytes]], Optional[BaseException]], None]


class BatchPipeline:
    def __init__(self, engine: Engine, device_fn: Callable, on_batch: Optional[Callable] = None):
        """``device_fn(job)`` runs the device stage (the batcher's wrapper adds the CPU fallback);
        ``on_batch(n_requests, seconds)`` observes each finished batch."""
        self.engine = engine
        self._device_fn = device_fn
        self._on_batch = on_batch
        self._dq: "queue.SimpleQueue" = queue.SimpleQueue()
        self._eq: "queue.SimpleQueue" = queue.SimpleQueue()
        self._lock = threading.Lock()
        self._inflight = 0
        self.submitted = 0              # batches that went through the threads (not inline)
        self.timeline: Optional[list] = None   # set to [] to record (stage, batch size, start, end)
        # busy seconds per stage (and batches / requests through them): the serving breakdown
        # (/admin/stages, benchmarks/bench_configs.py concurrent_http)
        self.stage_s = {"pack": 0.0, "device": 0.0, "emit": 0.0, "complete": 0.0}
        self.batches = 0
        self.requests = 0
        self._threads = [threading.Thread(target=self._device_loop, name="lp-pipe-device", daemon=True),
                         threading.Thread(target=self._emit_loop, name="lp-pipe-emit", daemon=True)]
        for t in self._threads:
            t.start()

    def idle(self) -> bool:
        """No batch in flight. Only the producer adds batches, so an idle pipeline seen by the
        producer stays idle until it submits: it may then run a batch inline, with no hand-off."""
        return self._inflight == 0

    def run_inline(self, logs: Sequence) -> List[bytes]:
        """All three stages on the calling thread (lowest latency for a lone batch)."""
        assert self.idle(), "inline batch while the pipeline is busy would reorder frequency updates"
        t0 = time.perf_counter()
        job = self.engine.pack_batch(logs, early_upload=True)
        try:
            t1 = time.perf_counter()
            self._device_fn(job)
            t2 = time.perf_counter()
            outs = self.engine.emit_batch(job)
        finally:
            self.engine.release_batch(job)
        t3 = time.perf_counter()
        st = self.stage_s
        st["pack"] += t1 - t0
        st["device"] += t2 - t1
        st["emit"] += t3 - t2
        self.batches += 1
        self.requests += len(logs)
        if self._on_batch:
            self._on_batch(len(logs), t3 - t0)
        return outs

    def submit(self, logs: Sequence, done: Done) -> None:
        """Pack on the calling thread (blocks while 3 batches are in flight), then hand over."""
        t0 = time.perf_counter()
        try:
            job = self.engine.pack_batch(logs)
        except Exception as e:  # noqa: BLE001
            log.exception("batch packing failed")
            done(None, e)
            return
        t1 = time.perf_counter()
        self.stage_s["pack"] += t1 - t0
        if self.timeline is not None:
            self.timeline.append(("pack", len(logs), t0, t1))
        with self._lock:
            self._inflight += 1
            self.submitted += 1
        self._dq.put((job, done, t0))

    def _device_loop(self) -> None:
        from ..utils.threadsample import set_os_thread_name
        set_os_thread_name("lp-pipe-device")
        eng = self.engine
        if eng.device.type == "cuda":
            torch.cuda.set_device(eng.device)
        while True:
            item = self._dq.get()
            if item is None:
                self._eq.put(None)
                return
            job, done, t0 = item
            try:
                ts = time.perf_counter()
                self._device_fn(job)
                te = time.perf_counter()
                self.stage_s["device"] += te - ts
                if self.timeline is not None:
                    self.timeline.append(("device", len(job.logs), ts, te))
                self._eq.put(item)
            except Exception as e:  # noqa: BLE001
                log.exception("batch failed")
                self._finish(job, done, None, e, t0)

    def _emit_loop(self) -> None:
        from ..utils.threadsample import set_os_thread_name
        set_os_thread_name("lp-pipe-emit")
        while True:
            item = self._eq.get()
            if item is None:
                return
            job, done, t0 = item
            try:
                ts = time.perf_counter()
                outs = self.engine.emit_batch(job)
                te = time.perf_counter()
                self.stage_s["emit"] += te - ts
                if self.timeline is not None:
                    self.timeline.append(("emit", len(job.logs), ts, te))
            except Exception as e:  # noqa: BLE001
                log.exception("response emission failed")
                self._finish(job, done, None, e, t0)
                continue
            self._finish(job, done, outs, None, t0)

    def _finish(self, job, done: Done, outs, exc, t0: float) -> None:
        self.engine.release_batch(job)
        with self._lock:
            self._inflight -= 1
        if outs is not None and self._on_batch:
            self._on_batch(len(job.logs), time.perf_counter() - t0)
        ts = time.perf_counter()
        try:
            done(outs, exc)
        except Exception:  # noqa: BLE001
            log.exception("batch completion callback failed")
        te = time.perf_counter()
        self.stage_s["complete"] += te - ts
        self.batches += 1
        self.requests += len(job.logs)
        if self.timeline is not None:
            self.timeline.append(("complete", len(job.logs), ts, te))

    def close(self) -> None:
        self._dq.put(None)
        for t in self._threads:
            t.join(timeout=5)
