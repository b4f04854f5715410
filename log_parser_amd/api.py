"""High-level Python API (what the reference exposes only over HTTP, Parse.java / AnalysisService)."""
from __future__ import annotations

import json
from typing import List, Optional, Sequence

import torch

from .engine import Engine, resolve_device
from .frequency import FrequencyState
from .models.compiled import CompiledLibrary
from .models.library import load_pattern_directory
from .models.schema import PatternSet
from .utils.config import Config


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

    @classmethod
    def from_directory(cls, directory: str, **kw) -> "LogParser":
        return cls(load_pattern_directory(directory), **kw)

    def parse(self, logs: str) -> dict:
        return json.loads(self.engine.analyze_json(logs))

    def parse_json(self, logs: str) -> bytes:
        return self.engine.analyze_json(logs)

    def parse_batch(self, logs: Sequence[str]) -> List[dict]:
        return [json.loads(x) for x in self.engine.analyze_batch_json(list(logs))]

    def parse_stream(self, data, chunk_bytes: Optional[int] = None, topk: int = 100, keep_events: bool = False):
        from .parallel.stream import StreamAnalyzer
        return StreamAnalyzer(self.engine, chunk_bytes=chunk_bytes, topk=topk, keep_events=keep_events).run(data)

    @property
    def frequency(self) -> FrequencyState:
        return self.engine.freq
