"""In-process API: the engine embedded in a Python program, without the HTTP front end.

The reference exposes its analysis only through ``POST /parse`` (``Parse.java:41-61`` ->
``AnalysisService.analyze``) and keeps ``FrequencyTrackingService``'s statistics / reset methods
internal (``FrequencyTrackingService.java:101-134``). :class:`LogParser` offers the same analysis
to embedders, with what an in-process user needs beyond one call at a time:

* ``parse`` / ``parse_json``: one document, synchronously (the AnalysisResult dict / JSON bytes);
* ``submit``: thread-safe asynchronous analysis through the same continuous batcher the service
  uses (concurrent callers share device batches; the frequency window sees them in submission
  order) -- ``Future`` of the JSON bytes;
* ``parse_file``: a log file of any size -- whole-document analysis below the stream threshold,
  otherwise an mmap'd chunked stream (summary + top-k, bounded memory);
* ``load_resident`` / ``analyze_resident``: a multi-GB log held in HBM and re-analysed (with this
  or another parser's library) without crossing PCIe again;
* ``validate``: the library's compile report (regex kinds, invalid / host-fallback regexes) that
  the reference would only discover as HTTP 500s, request by request (AnalysisService.java:64);
* the frequency-tracking surface: ``pattern_frequency``, ``frequency_statistics``,
  ``reset_pattern_frequency``, ``reset_all_frequencies``.
"""
from __future__ import annotations

import json
import mmap
import os
import threading
from concurrent.futures import Future
from typing import List, Optional, Sequence

from .engine import Engine, resolve_device
from .frequency import FrequencyState
from .models.compiled import KIND_DFA, KIND_FALLBACK, KIND_INVALID, KIND_NFA, CompiledLibrary
from .models.library import load_pattern_directory
from .models.schema import PatternSet
from .utils.config import Config

_KIND_NAMES = {KIND_DFA: "dfa", KIND_NFA: "nfa", KIND_FALLBACK: "host-fallback", KIND_INVALID: "invalid"}


class LogParser:
    """``LogParser.from_directory(dir).parse(logs)`` -> AnalysisResult dict."""

    def __init__(self, pattern_sets: List[PatternSet], config: Optional[Config] = None,
                 device: Optional[str] = None, freq: Optional[FrequencyState] = None):
        self.config = config or Config.load()
        dev = resolve_device(device or self.config["engine.device"])
        self.library = CompiledLibrary(pattern_sets, self.config.scoring,
                                       max_dfa_states=int(self.config["engine.dfa-max-states"]),
                                       nfa_engine=str(self.config["engine.nfa-engine"]))
        self.engine = Engine(self.library, self.config, device=dev, freq=freq)
        self._batcher = None
        self._lock = threading.Lock()

    @classmethod
    def from_directory(cls, directory: str, **kw) -> "LogParser":
        return cls(load_pattern_directory(directory), **kw)

    # ---- analysis -----------------------------------------------------------------------------
    def parse(self, logs: str) -> dict:
        return json.loads(self.parse_json(logs))

    def parse_json(self, logs: str) -> bytes:
        if self._batcher is not None:         # the batcher owns the engine now: go through it
            return self._batcher.submit(logs).result()
        with self._lock:                      # the engine's staging buffers serve one batch at a time
            return self.engine.analyze_json(logs)

    def parse_batch(self, logs: Sequence[str]) -> List[dict]:
        """Several documents as ONE device batch (each keeps its own line numbering / N)."""
        with self._lock:
            return [json.loads(x) for x in self.engine.analyze_batch_json(list(logs))]

    def submit(self, logs: str) -> "Future[bytes]":
        """Asynchronous, thread-safe: the request joins the continuous batcher (serve/app.py) --
        concurrent submitters share device batches, in submission order."""
        if self._batcher is None:
            with self._lock:
                if self._batcher is None:
                    from .serve.app import Batcher
                    from .utils.metrics import Metrics
                    c = self.config
                    self._batcher = Batcher(self.engine, int(c["engine.batch.max-requests"]),
                                            int(c["engine.batch.max-bytes"]), float(c["engine.batch.max-wait-ms"]),
                                            Metrics())
        return self._batcher.submit(logs)

    def stream_threshold(self) -> int:
        """File size above which ``parse_file`` streams (StreamResult summary) instead of analysing
        one whole document (full AnalysisResult): ``engine.stream.threshold-bytes``, independent of
        the HBM-sized stream chunk, so the output format and host memory of a file do not depend
        on the GPU it runs on."""
        return int(self.config["engine.stream.threshold-bytes"])

    def parse_stream(self, data, chunk_bytes: Optional[int] = None, topk: int = 100, keep_events: bool = False):
        from .parallel.stream import StreamAnalyzer
        with self._lock:
            return StreamAnalyzer(self.engine, chunk_bytes=chunk_bytes, topk=topk, keep_events=keep_events).run(data)

    def parse_file(self, path: str, stream: Optional[bool] = None, topk: int = 20, raw: bool = False):
        """A log file: the AnalysisResult dict (``raw``: its JSON bytes) when it is below the stream
        threshold (or ``stream=False``), else a ``StreamResult`` of an mmap'd chunked pass."""
        size = os.path.getsize(path)
        if stream is None:
            stream = size > self.stream_threshold()
        with open(path, "rb") as f:
            if not stream:
                text = f.read().decode("utf-8", errors="surrogateescape")
                return self.parse_json(text) if raw else self.parse(text)
            mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
            try:
                return self.parse_stream(mm, topk=topk)
            finally:
                if size:
                    mm.close()

    def load_resident(self, data, chunk_bytes: Optional[int] = None):
        """Stage ``data`` into HBM once (``parallel.stream.ResidentLog``) for repeated analyses."""
        from .parallel.stream import ResidentLog
        return ResidentLog.load(data, self.engine, chunk_bytes=chunk_bytes)

    def analyze_resident(self, resident, topk: int = 100, keep_events: bool = False):
        from .parallel.stream import StreamAnalyzer
        with self._lock:
            return StreamAnalyzer(self.engine, chunk_bytes=resident.chunk_bytes, topk=topk,
                                  keep_events=keep_events).run(resident)

    # ---- library report -----------------------------------------------------------------------
    def validate(self, allow=("nfa",)) -> dict:
        """Compile report: library counts plus every regex that is invalid, routed to the host
        fallback, or of a kind not in ``allow``."""
        problems = []
        for r in self.library.regexes:
            name = _KIND_NAMES.get(r.kind, str(r.kind))
            if r.kind in (KIND_INVALID, KIND_FALLBACK) or (r.kind == KIND_NFA and "nfa" not in allow):
                problems.append({"regex": r.pattern, "kind": name, "error": r.error, "roles": sorted(r.roles)})
        return {"library": self.library.summary(), "problems": problems}

    # ---- frequency tracking (FrequencyTrackingService.java:101-134) ---------------------------
    @property
    def frequency(self) -> FrequencyState:
        return self.engine.freq

    def pattern_frequency(self, pattern_id: str) -> Optional[dict]:
        return self.engine.freq.get_pattern_frequency(pattern_id)

    def frequency_statistics(self) -> dict:
        return self.engine.freq.statistics()

    def reset_pattern_frequency(self, pattern_id: str) -> None:
        self.engine.freq.reset(pattern_id)

    def reset_all_frequencies(self) -> None:
        self.engine.freq.reset_all()

    def close(self) -> None:
        if self._batcher is not None:
            self._batcher.close()
            self._batcher = None
