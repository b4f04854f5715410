"""Pure-Python golden model of the reference analysis pipeline (the test oracle).

A line-by-line re-statement of the reference's *semantics*, kept deliberately naive and
independent of the device engine (SURVEY §4, §7 phase 0). Every quirk is reproduced:

* line split ``logs.split("\\r?\\n")`` with Java trailing-empty removal (``AnalysisService.java:53``)
* event order: line, then pattern-set order, then pattern order (``AnalysisService.java:89-113``)
* context extraction, ``[i,i]`` only when rules are null (``AnalysisService.java:132-156``)
* 7-factor score, left-to-right product (``ScoringService.java:63-112``)
* chronological piecewise-linear factor (``ScoringService.java:123-151``)
* proximity: nearest secondary hit within ``min(maxWindow, proximityWindow)``, self line
  excluded, ``1 + Σ w·exp(-d/decay)`` (``ScoringService.java:161-190,315-347``)
* temporal: last event within ±5 (inclusive of i), earlier events by nearest hit strictly
  before a cursor that starts at i, unbounded backwards (``ScoringService.java:199-305``)
* context factor with ERR/WARN else-if, stack bonus, density penalty, cap
  (``ContextAnalysisService.java:46-117``)
* frequency penalty computed *before* recording the match (``ScoringService.java:84-88``,
  ``FrequencyTrackingService.java:41-93``)
* summary with ``NONE`` on empty and first-wins ties (``AnalysisService.java:188-215``)
"""
from __future__ import annotations

import math
import re
import threading
import time
import uuid
from collections import deque
from datetime import datetime, timezone
from typing import Callable, Dict, List, Optional, Sequence

from .models.schema import Pattern, PatternSet, pattern_to_json
from .regex.javacompat import compile_java
from .utils.config import ScoringParams

SEVERITY_MULTIPLIERS = {"CRITICAL": 5.0, "HIGH": 3.0, "MEDIUM": 2.0, "LOW": 1.5, "INFO": 1.0}
SEVERITY_ORDER = ["INFO", "LOW", "MEDIUM", "HIGH", "CRITICAL"]

ERROR_RE = r"(?i)\b(ERROR|FATAL|CRITICAL|SEVERE)\b"
WARN_RE = r"(?i)\b(WARN|WARNING)\b"
STACK_RE = r"^\s*at\s+[\w\.\$]+\(.*\)\s*$"
EXC_RE = r"\b\w*Exception\b|\b\w*Error\b"
CONTEXT_REGEXES = (ERROR_RE, WARN_RE, STACK_RE, EXC_RE)

_SPLIT = re.compile(r"\r?\n")



def java_blank(pid) -> bool:
    """``id == null || id.trim().isEmpty()`` (FrequencyTrackingService.java:42,65). Java's
    String.trim() strips every char <= U+0020 (controls included) and nothing else: "\x01" is
    blank, a non-breaking space (U+00A0) or "\u2003" is not -- unlike Python's str.strip()."""
    return pid is None or all(ord(c) <= 0x20 for c in pid)

def split_lines(logs: str) -> List[str]:
    """Java ``String.split("\\r?\\n")`` (limit 0)."""
    if _SPLIT.search(logs) is None:
        return [logs]
    parts = _SPLIT.split(logs)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def severity_key(sev: Optional[str]) -> str:
    return (sev or "").upper()


class FrequencyTracker:
    """Sliding-window match counter per pattern id (``FrequencyTrackingService.java:20-162``).

    ``PatternFrequency`` lives in the unavailable common-lib; semantics follow SURVEY §2.4:
    ``hourlyRate = #matches within the last W hours / W``.
    """

    def __init__(self, params: ScoringParams, clock: Callable[[], float] = time.time):
        self.params = params
        self.clock = clock
        self._ts: Dict[str, deque] = {}
        self._lock = threading.Lock()

    def _prune(self, dq: deque, now: float) -> None:
        horizon = now - self.params.freq_window_hours * 3600.0
        while dq and dq[0] <= horizon:
            dq.popleft()

    def record(self, pid: Optional[str]) -> None:
        if java_blank(pid):
            return
        with self._lock:
            self._ts.setdefault(pid, deque()).append(self.clock())

    def count(self, pid: str) -> int:
        with self._lock:
            dq = self._ts.get(pid)
            if dq is None:
                return 0
            self._prune(dq, self.clock())
            return len(dq)

    def hourly_rate(self, pid: str) -> float:
        return self.count(pid) / float(self.params.freq_window_hours)

    def penalty(self, pid: Optional[str]) -> float:
        if java_blank(pid):
            return 0.0
        with self._lock:
            if pid not in self._ts:
                return 0.0
        rate = self.hourly_rate(pid)
        thr = self.params.freq_threshold
        if rate <= thr:
            return 0.0
        return min(self.params.freq_max_penalty, (rate - thr) / thr)

    def statistics(self) -> Dict[str, int]:
        return {k: self.count(k) for k in list(self._ts)}

    def reset(self, pid: str) -> None:
        with self._lock:
            if pid in self._ts:
                self._ts[pid].clear()

    def reset_all(self) -> None:
        with self._lock:
            self._ts.clear()


def _find(regex: Optional[str], line: str) -> bool:
    if regex is None:
        return False
    return compile_java(regex).search(line) is not None


def chronological_factor(line_index: int, n_lines: int, p: ScoringParams) -> float:
    pos = float(line_index) / n_lines
    e, t = p.early_bonus_threshold, p.penalty_threshold
    if pos <= e:
        return 1.5 + (e - pos) * ((p.max_early_bonus - 1.5) / e)
    if pos <= t:
        return 1.0 + (t - pos) * (0.5 / (t - e))
    return 0.5 + (1.0 - pos)


def proximity_factor(pattern: Pattern, i: int, lines: Sequence[str], p: ScoringParams) -> float:
    secs = pattern.secondary_patterns
    if not secs:
        return 1.0
    total = 0.0
    n = len(lines)
    for s in secs:
        w = min(p.max_window, s.proximity_window)
        start, end = max(0, i - w), min(n, i + w + 1)
        best = -1.0
        for j in range(start, end):
            if j == i:
                continue
            if _find(s.regex, lines[j]):
                d = float(abs(j - i))
                if best < 0 or d < best:
                    best = d
        if best >= 0:
            total += s.weight * math.exp(-best / p.decay_constant)
    return 1.0 + total


def _sequence_matched(seq, i: int, lines: Sequence[str]) -> bool:
    events = seq.events
    if not events:
        return False
    n = len(lines)
    cursor = 0
    for k in range(len(events) - 1, -1, -1):
        rx = events[k].regex
        if k == len(events) - 1:
            start, end = max(0, i - 5), min(n, i + 5 + 1)
            if not any(_find(rx, lines[j]) for j in range(start, end)):
                return False
            cursor = i
        else:
            found = -1
            for j in range(cursor - 1, -1, -1):
                if _find(rx, lines[j]):
                    found = j
                    break
            if found < 0:
                return False
            cursor = found
    return True


def temporal_factor(pattern: Pattern, i: int, lines: Sequence[str]) -> float:
    seqs = pattern.sequence_patterns
    if not seqs:
        return 1.0
    total = 0.0
    for s in seqs:
        if _sequence_matched(s, i, lines):
            total += s.bonus_multiplier
    return 1.0 + total


def context_factor(ctx_lines: Optional[List[str]], p: ScoringParams) -> float:
    if not ctx_lines:
        return 1.0
    score = 0.0
    err = stack = 0
    for line in ctx_lines:
        if _find(ERROR_RE, line):
            err += 1
            score += 0.4
        elif _find(WARN_RE, line):
            score += 0.2
        if _find(STACK_RE, line):
            stack += 1
            score += 0.1
        if _find(EXC_RE, line):
            score += 0.3
    if stack > 0:
        score += min(stack * 0.1, 0.5)
    total = len(ctx_lines)
    if total > 10 and (stack + err) > total * 0.7:
        score *= 0.8
    f = 1.0 + score
    if f > p.max_context_factor:
        f = p.max_context_factor
    return f


def extract_context(lines: Sequence[str], i: int, rules) -> dict:
    ctx = {"matchedLine": lines[i], "linesBefore": None, "linesAfter": None}
    if rules is None:
        return ctx
    before = max(0, rules.lines_before)
    after = max(0, rules.lines_after)
    ctx["linesBefore"] = list(lines[max(0, i - before):i])
    ctx["linesAfter"] = list(lines[i + 1:min(len(lines), i + 1 + after)])
    return ctx


def _ctx_lines(ctx: dict) -> List[str]:
    out: List[str] = []
    if ctx["linesBefore"] is not None:
        out.extend(ctx["linesBefore"])
    if ctx["matchedLine"] is not None:
        out.append(ctx["matchedLine"])
    if ctx["linesAfter"] is not None:
        out.extend(ctx["linesAfter"])
    return out


def score_event(pattern: Pattern, i: int, lines: Sequence[str], ctx: dict,
                p: ScoringParams, freq: FrequencyTracker) -> float:
    conf = pattern.primary_pattern.confidence
    sev = SEVERITY_MULTIPLIERS.get(severity_key(pattern.severity), 1.0)
    chrono = chronological_factor(i, len(lines), p)
    prox = proximity_factor(pattern, i, lines, p)
    temp = temporal_factor(pattern, i, lines)
    ctxf = context_factor(_ctx_lines(ctx), p)
    pen = freq.penalty(pattern.id)
    freq.record(pattern.id)
    return conf * sev * chrono * prox * temp * ctxf * (1.0 - pen)


def build_summary(events: List[dict]) -> dict:
    if not events:
        return {"significantEvents": 0, "highestSeverity": "NONE", "severityDistribution": {}}
    dist: Dict[str, int] = {}
    best = None
    best_idx = -2
    for e in events:
        s = severity_key(e["matchedPattern"].get("severity"))
        dist[s] = dist.get(s, 0) + 1
        idx = SEVERITY_ORDER.index(s) if s in SEVERITY_ORDER else -1
        if idx > best_idx:
            best_idx, best = idx, s
    return {"significantEvents": len(events), "highestSeverity": best, "severityDistribution": dist}


def analyze(logs: str, pattern_sets: List[PatternSet], params: ScoringParams,
            freq: FrequencyTracker) -> dict:
    """``AnalysisService.analyze`` (``AnalysisService.java:50-122``)."""
    t0 = time.time()
    lines = split_lines(logs)
    events: List[dict] = []
    for li, line in enumerate(lines):
        for ps in pattern_sets:
            for pat in (ps.patterns or []):
                if pat.primary_pattern is None or not _find(pat.primary_pattern.regex, line):
                    continue
                ctx = extract_context(lines, li, pat.context_extraction)
                sc = score_event(pat, li, lines, ctx, params, freq)
                events.append({"lineNumber": li + 1, "matchedPattern": pattern_to_json(pat),
                               "context": ctx, "score": sc})
    meta = {
        "processingTimeMs": int((time.time() - t0) * 1000),
        "totalLines": len(lines),
        "analyzedAt": datetime.now(timezone.utc).isoformat().replace("+00:00", "Z"),
        "patternsUsed": [(ps.metadata.library_id if ps.metadata else None) for ps in pattern_sets],
    }
    return {"analysisId": str(uuid.uuid4()), "metadata": meta, "events": events,
            "summary": build_summary(events)}
