"""Dotted-key configuration system (MicroProfile-Config compatible key names).

Reference parity: the reference reads 10 keys through ``@ConfigProperty`` with in-code
defaults that mirror ``src/main/resources/application.properties:1-20``
(``PatternService.java:35-36``, ``ScoringService.java:38-51``,
``ContextAnalysisService.java:24``, ``FrequencyTrackingService.java:27-34``).

Resolution order (highest wins), same as MicroProfile Config ordinals:
  1. explicit overrides (``-Dkey=value`` on the CLI, or ``Config(overrides=...)``)
  2. environment variables, MicroProfile mapping: ``scoring.proximity.max-window`` is also
     looked up as ``SCORING_PROXIMITY_MAX_WINDOW`` (non-alphanumerics -> ``_``, upper-cased)
  3. an ``application.properties`` file (``LP_CONFIG`` env var or ``config/application.properties``)
  4. in-code defaults below.

New keys live under ``engine.*`` (device / parallel / batching knobs) and ``server.*``.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, Mapping, Optional

# key -> (default, type)
REFERENCE_KEYS: Dict[str, tuple] = {
    "pattern.directory": ("/shared/patterns", str),
    "scoring.proximity.decay-constant": (10.0, float),
    "scoring.proximity.max-window": (100, int),
    "scoring.chronological.early-bonus-threshold": (0.2, float),
    "scoring.chronological.max-early-bonus": (2.5, float),
    "scoring.chronological.penalty-threshold": (0.5, float),
    "scoring.context.max-context-factor": (2.5, float),
    "scoring.frequency.threshold": (10.0, float),
    "scoring.frequency.max-penalty": (0.8, float),
    "scoring.frequency.time-window-hours": (1, int),
}

ENGINE_KEYS: Dict[str, tuple] = {
    # "auto" -> cuda if available else cpu. "cuda" fails loudly without the HIP extension.
    "engine.device": ("auto", str),
    # data-parallel serving: "" = engine.device only, "all" = every visible GPU, or "cuda:0,cuda:1"
    "engine.serve-devices": ("", str),
    # engines on OTHER GPUs share the first engine's HBM frequency window over xGMI peer access
    # (off: they share one host window; streams of the same GPU always share the device window)
    "engine.serve.peer-window": (False, bool),
    # bytes per streamed H2D chunk for long logs (double-buffered pinned staging); 0 = sized from
    # the GPU's free HBM (parallel/stream.py auto_chunk_bytes: 1/16 of it, 256 MiB .. 8 GiB)
    "engine.chunk-bytes": (0, int),
    # LogParser.parse_file / CLI: files above this many bytes are streamed (StreamResult summary +
    # top-k); smaller files are analysed as one document (full AnalysisResult)
    "engine.stream.threshold-bytes": (256 << 20, int),
    # capacity hint for candidate (line, regex) pairs per chunk; grown on overflow
    "engine.candidate-capacity": (1 << 22, int),
    # max DFA states per regex before it is routed to the NFA engine
    "engine.dfa-max-states": (2048, int),
    # NFA engine of regexes whose DFA blows up: "bpg" (bit-parallel Glushkov programs, literal
    # prefilter candidates or every line) or "mfma" (state-transition GEMM, every line, <= 64
    # positions; A/B engine)
    "engine.nfa-engine": ("bpg", str),
    # context-feature engine: "mfma" (NFA state-transition GEMM on matrix cores) or "dfa"
    "engine.context-engine": ("dfa", str),
    # run the literal-free scan engines on a second HIP stream, overlapping the literal prefilter
    # (off: the cross-stream event wait cost more than the overlap saved -- 10k-line request
    # 0.362 -> 0.382-0.408 ms on the MI355X box, tools/engine_phases.py A/B)
    "engine.scan-stream": (False, bool),
    # bulk / document steps: the early literal prefilter on its own HIP stream, beside the rest of
    # the line index and the literal-free scans (prefilter_early; config 2's chains overlap)
    "engine.prefilter-stream": (True, bool),
    # bulk steps: fold the line index's first pass into the literal prefilter (one read of the text
    # fewer; opt-in until a GPU A/B is in)
    "engine.fused-line-index": (False, bool),
    # the device half of a batch in one native call (csrc/runtime/request.cpp) when applicable
    "engine.native-runner": (True, bool),
    # runner, request-sized batches: events / score / frequency record read the matcher counts on
    # the device (no mid-batch host read; the record is gated on the capacities holding) and
    # k_publish writes the counters + compacted results into pinned host memory (no copies back):
    # 10k-line request GPU span 352 -> 326 us, engine p50 0.310 -> 0.302 ms (profiles/r2_v10)
    "engine.runner-device-counts": (True, bool),
    # backtracker side path (ops/side_path.py): the GPU's first wall-clock wait for the host's
    # verified keys (k_wait_host); a timeout re-runs that step on the host-verified path and doubles it
    "engine.side-path-wait-s": (2.0, float),
    # serve a batch from the CPU backend when the device path fails (availability)
    "engine.fallback-cpu": (True, bool),
    # per-stage HIP-event timers, reported in response metadata as stageTimingsMs (opt-in)
    "engine.trace": (False, bool),
    # fault injection for tests: fail the device path every N-th batch (0 = off)
    "engine.fault-inject-every": (0, int),
    # fault injection for tests: fail every N-th batch AFTER its frequency record (0 = off)
    "engine.fault-inject-after-record": (0, int),
    # continuous batching
    "engine.batch.max-requests": (2048, int),
    "engine.batch.max-bytes": (256 << 20, int),
    # serving: size the pinned batch stages for this many bytes at start-up (capped by max-bytes;
    # 0 = grow on demand). Default = max-bytes: no batch ever grows a stage. A growth pins a new
    # buffer (~30 ms for 200+ MB) while holding the GIL, which stalls every Python stage of the
    # pipeline; in the config-5 burst the first 1,800-2,048-request batches hit it (profiles/r4_d)
    "engine.batch.prewarm-bytes": (256 << 20, int),
    # extra wait for more requests after the first one; 0 = greedy continuous batching (a batch
    # forms from whatever queued while the previous one ran; an idle server answers at once)
    "engine.batch.max-wait-ms": (0.0, float),
    # top-k events kept by the distributed reduction (0 = all events)
    "engine.topk": (100, int),
    # keep the sliding-window frequency state in HBM when one engine owns a GPU (K8)
    "engine.frequency.device-resident": (True, bool),
    # persist frequency state (snapshot path, empty = disabled, reference default)
    "engine.frequency.snapshot-path": ("", str),
    # max request body (reference: Quarkus default 10 MiB)
    "server.max-body-bytes": (1 << 30, int),
    "server.port": (8080, int),
    "server.host": ("0.0.0.0", str),
    # HTTP front end: "native" (C++ epoll server, csrc/io/http_server.cpp) or "uvicorn" (FastAPI)
    "server.http": ("native", str),
    # native front end IO threads (epoll loops receiving / validating bodies, sending responses);
    # 0 = auto: half this process's CPU budget, 2..8 (tools/http_ceiling.py: the config-5 burst with no
    # engine reaches 13.7k req/s with 2 threads, 32k with 8, on an 8-CPU container)
    "server.io-threads": (0, int),
    # serving processes (serve/procs.py): 1 = this process only; N > 1 = N processes started before
    # any GPU call, each with its own SO_REUSEPORT listeners, GIL and pipeline, sharing ONE
    # frequency window (host shared memory) in arrival-ticket order; -1 = one per visible GPU.
    # Process i serves on engine.serve-devices[i % n] (or engine.device when that is empty)
    "server.processes": (1, int),
    # serving processes: restarts of one dead worker before the supervisor stops the group (the
    # others keep serving meanwhile)
    "server.max-restarts": (3, int),
    # single-GPU service: bind the process to the CPUs of the GPU's NUMA node (serve/__main__.py)
    "server.numa-bind": (True, bool),
    # native front end: close keep-alive connections idle this long (no request in flight)
    "server.idle-timeout-s": (60.0, float),
    # native front end over a GPU engine: start the IO threads, the pump and the decode helper on one
    # hardware thread per core of ONE last-level cache (a CCD): a body received by an IO thread is
    # decoded by the helper and packed by the pump (a lone-body A/B was within run-to-run spread,
    # profiles/r6_d; on SMT siblings the receiving and the decoding thread share a core)
    "server.l3-affinity": (True, bool),
    # native front end: a POST /parse body of >= 64 KiB has its `logs` string validated and decoded
    # by the IO thread between reads while it arrives; the final parse resumes there (csrc/io/json_in.h
    # LogsPrefetch). The request's verdict (400 / 200) is still the final parse's.
    "server.prefetch-logs": (True, bool),
    # native front end over a GPU engine: up to this many pinned (page-locked) buffers receive the
    # decoded logs of bodies >= 256 KiB; the engine stages such a request in place (no copy of the
    # text into its own stage, and the decoder's newline positions replace the packer's scan:
    # /parse p50 0.42-0.43 -> 0.40 ms, profiles/r6_e). 0: pageable buffers, copied.
    "server.pinned-decode-buffers": (8, int),
    # native front end: an IO thread decodes a /parse body's `logs` string itself (bodies >= 4 KiB)
    # only while it holds at most this many connections; under a burst the bodies reach the packer
    # undecoded and the IO threads only receive and validate. -1: always decode on the IO thread.
    "server.io-decode-max-conns": (64, int),
    # native front end: IO threads poll this long after activity before sleeping in epoll_wait
    "server.io-spin-us": (0.0, float),
    # native front end: the pump polls for the next request this long before sleeping on the queue
    # (a sleeping pump took ~45 us to wake, tools/parse_tail.py)
    "server.pump-spin-us": (1000.0, float),
    # TCP_QUICKACK on every read (delayed ACKs stalled ~1-2% of 1 MB bodies by ~1.5 ms)
    "server.tcp-quickack": (True, bool),
    # SO_RCVBUF of accepted sockets (0 = kernel autotuning)
    "server.rcvbuf-bytes": (0, int),
    # per-request receive / validate / queue / engine microseconds on stderr (tools/parse_tail.py)
    "server.trace-requests": (False, bool),
    # record the serving pipeline's per-batch stage intervals (pack / device / emit / complete),
    # returned by GET /admin/stages (benchmarks/bench_configs.py concurrent_http --timeline)
    "server.stage-timeline": (False, bool),
    # freeze the startup heap + raise GC thresholds in the batching server (submit-path latency)
    "server.gc-tuning": (True, bool),
    # Python GIL switch interval in the serving process (ms; 0 = interpreter default 5 ms). The
    # pipeline's device thread needs the GIL for every launch; a short interval keeps it from
    # waiting behind the pack / emit threads' Python work
    "server.switch-interval-ms": (0.0, float),
    # reference logs one INFO line per match (AnalysisService.java:96-99); we log it at DEBUG
    "server.log-matches": (False, bool),
}

ALL_KEYS: Dict[str, tuple] = {**REFERENCE_KEYS, **ENGINE_KEYS}


def env_name(key: str) -> str:
    """MicroProfile Config env-var mapping: non-alphanumerics -> '_', upper-case."""
    return re.sub(r"[^A-Za-z0-9]", "_", key).upper()


def _coerce(value: Any, typ: type) -> Any:
    if typ is bool:
        if isinstance(value, bool):
            return value
        return str(value).strip().lower() in ("1", "true", "yes", "on")
    if typ is int:
        return int(float(value)) if isinstance(value, str) and "." in value else int(value)
    return typ(value)


def parse_properties(text: str) -> Dict[str, str]:
    """Minimal java.util.Properties parser (key=value / key: value, # and ! comments)."""
    out: Dict[str, str] = {}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line[0] in "#!":
            continue
        m = re.match(r"([^=:\s]+)\s*[=:\s]\s*(.*)$", line)
        if m:
            out[m.group(1)] = m.group(2).strip()
    return out


TOPK_MAX = 1024     # rows the summary / top-k kernel keeps (ops/kernels.py SUMMARY_MAX_K)


def _validate(v: Mapping[str, Any]) -> None:
    k = v.get("engine.topk")
    if k is not None and not 0 <= int(k) <= TOPK_MAX:
        raise ValueError(f"engine.topk must be within [0, {TOPK_MAX}], got {k}")
    e = v.get("engine.nfa-engine")
    if e is not None and e not in ("bpg", "mfma"):
        raise ValueError(f"engine.nfa-engine must be 'bpg' or 'mfma', got {e!r}")


@dataclass(frozen=True)
class Config:
    values: Mapping[str, Any] = field(default_factory=dict)

    @staticmethod
    def load(overrides: Optional[Mapping[str, Any]] = None,
             properties_path: Optional[str] = None,
             environ: Optional[Mapping[str, str]] = None) -> "Config":
        environ = os.environ if environ is None else environ
        vals: Dict[str, Any] = {k: d for k, (d, _) in ALL_KEYS.items()}
        path = properties_path or environ.get("LP_CONFIG") or os.path.join("config", "application.properties")
        if path and os.path.isfile(path):
            with open(path, "r", encoding="utf-8") as f:
                for k, v in parse_properties(f.read()).items():
                    vals[k] = v
        for k in ALL_KEYS:
            e = env_name(k)
            if e in environ:
                vals[k] = environ[e]
        if overrides:
            for k, v in overrides.items():
                vals[k] = v
        typed = {}
        for k, v in vals.items():
            typ = ALL_KEYS[k][1] if k in ALL_KEYS else str
            typed[k] = _coerce(v, typ)
        _validate(typed)
        return Config(values=typed)

    def __getitem__(self, key: str) -> Any:
        return self.values[key]

    def get(self, key: str, default: Any = None) -> Any:
        return self.values.get(key, default)

    def with_overrides(self, **kv: Any) -> "Config":
        d = dict(self.values)
        for k, v in kv.items():
            d[k.replace("__", ".").replace("_", "-")] = v
        return Config(values=d)

    def replace(self, mapping: Mapping[str, Any]) -> "Config":
        d = dict(self.values)
        for k, v in mapping.items():
            typ = ALL_KEYS[k][1] if k in ALL_KEYS else type(v)
            d[k] = _coerce(v, typ)
        return Config(values=d)

    # ---- typed views used by the scoring code -------------------------------------------
    @property
    def scoring(self) -> "ScoringParams":
        return ScoringParams(
            decay_constant=float(self["scoring.proximity.decay-constant"]),
            max_window=int(self["scoring.proximity.max-window"]),
            early_bonus_threshold=float(self["scoring.chronological.early-bonus-threshold"]),
            max_early_bonus=float(self["scoring.chronological.max-early-bonus"]),
            penalty_threshold=float(self["scoring.chronological.penalty-threshold"]),
            max_context_factor=float(self["scoring.context.max-context-factor"]),
            freq_threshold=float(self["scoring.frequency.threshold"]),
            freq_max_penalty=float(self["scoring.frequency.max-penalty"]),
            freq_window_hours=int(self["scoring.frequency.time-window-hours"]),
        )


@dataclass(frozen=True)
class ScoringParams:
    decay_constant: float = 10.0
    max_window: int = 100
    early_bonus_threshold: float = 0.2
    max_early_bonus: float = 2.5
    penalty_threshold: float = 0.5
    max_context_factor: float = 2.5
    freq_threshold: float = 10.0
    freq_max_penalty: float = 0.8
    freq_window_hours: int = 1


def parse_cli_overrides(argv) -> Dict[str, str]:
    """Collect ``-Dkey=value`` arguments (Quarkus/MicroProfile style)."""
    out = {}
    for a in argv:
        if a.startswith("-D") and "=" in a:
            k, v = a[2:].split("=", 1)
            out[k] = v
    return out
