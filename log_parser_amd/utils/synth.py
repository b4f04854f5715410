"""Synthetic pod logs and randomly generated pattern libraries (BASELINE.json configs).

There is no network and the reference ships no fixtures, so tests and the bench
use generated data of the configured shape: ``n_patterns`` patterns (with secondary and
sequence patterns and context rules) and logs of ``n_lines`` realistic-looking lines into which
pattern triggers are planted at a controlled rate.
"""
from __future__ import annotations

import random
from typing import List, Optional, Tuple

from ..models.schema import PatternSet

LEVELS = ["INFO", "DEBUG", "WARN", "ERROR", "TRACE", "INFO", "INFO", "DEBUG"]
COMPONENTS = ["kubelet", "controller", "scheduler", "api-server", "etcd", "ingress", "app", "worker", "db-pool",
              "cache", "auth", "gateway"]
WORDS = ["request", "handled", "user", "session", "started", "completed", "processing", "batch", "queue", "item",
         "connection", "pool", "cache", "hit", "miss", "retry", "timeout", "latency", "bytes", "sent", "received",
         "config", "reload", "metrics", "flush", "checkpoint", "shard", "replica", "leader", "follower", "sync",
         "node", "pod", "container", "image", "pulled", "volume", "mounted", "probe", "ready", "healthy"]
SEVERITIES = ["CRITICAL", "HIGH", "MEDIUM", "LOW", "INFO"]
EXC = ["java.lang.NullPointerException", "java.io.IOException", "java.lang.IllegalStateException",
       "java.util.concurrent.TimeoutException", "java.lang.OutOfMemoryError"]


def _token(rng: random.Random, i: int) -> str:
    syl = ["ka", "ze", "tor", "vin", "qua", "mel", "dro", "pix", "lun", "sar", "bex", "fyr", "gol", "hup"]
    return "".join(rng.choice(syl) for _ in range(3)).capitalize() + str(i)


# letters that never start a 3-gram of the noise text (no vowels, no T/Z of the timestamps)
_CODE_LETTERS = "BCFGHJKMPQVWXY"


def _short_code(rng: random.Random, n: int) -> str:
    """3..6-byte error code (e.g. 'K42', 'QX7M1'): a short, realistic prefilter literal."""
    s = rng.choice(_CODE_LETTERS)
    while len(s) < n:
        s += rng.choice(_CODE_LETTERS + "0123456789")
    return s


def _literal_free(rng: random.Random, i: int) -> Tuple[str, str]:
    """A regex with no usable literal factor (every line must be scanned) + a matching sample.
    Parametrised by ``i`` so every regex of the library is a distinct string; shapes that the
    noise text of ``make_log`` never matches."""
    fam = i % 6
    a, b = 3 + (i // 6) % 3, 2 + (i // 18) % 6
    rx, sample = _literal_free_shape(rng, fam, a, b)
    if i >= 108:                     # past one cycle of shapes: an optional tail keeps them distinct
        rx += rf"(?:~{i // 108})?"
    return rx, sample


def _literal_free_shape(rng: random.Random, fam: int, a: int, b: int) -> Tuple[str, str]:
    up = "".join(rng.choice("ABCDEFGHJKLMNPQRSUVWXY") for _ in range(a + 1))
    dg = "".join(rng.choice("0123456789") for _ in range(b))
    if fam == 0:
        return rf"\b[A-Z]{{{a},}}_\d{{{b}}}\b", f"state {up}_{dg} entered"
    if fam == 1:
        return rf"\b[A-Z]{{2}}\d{{{a}}}[A-Z]{{{b}}}\b", \
            f"unit {up[:2]}{dg[:1] * a}{''.join(rng.choice('KMPQVX') for _ in range(b))} down"
    if fam == 2:
        m = 1 + b % 3
        return rf"\b\d{{1,3}}\.\d{{1,3}}\.\d{{{m},3}}\.\d+:\d{{{a + 1}}}\b", \
            f"peer 10.2.{'7' * m}.4:{'9' * (a + 1)} reset"
    if fam == 3:
        return rf"[^\s]+@[^\s]+\.[a-z]{{{b}}}\b", f"mail to ops@corp.{'x' * b} bounced"
    if fam == 4:
        return rf"\b[A-Z][a-z]+[A-Z][a-z]+\d{{{a}}}[A-Z]{{{b}}}\b", \
            f"got ShardLost{'5' * a}{'Q' * b} again"
    return rf"^\s+at\s+[a-z]+\.[A-Z]\w{{{a},}}\(\w*\.\w+:\d{{{b}}}\)", \
        f"\tat app.R{'x' * a}(Main.java:{'4' * b})"


def _bounded_gap(rng: random.Random, tok: str, i: int) -> Tuple[str, str, str, str]:
    """A bounded-gap regex (``X.{0,n}Y``: its DFA exceeds engine.dfa-max-states, so it runs as a
    bit-parallel Glushkov program) + a matching sample, and a bounded-gap secondary + its sample."""
    fam = i % 6
    g = (60, 80, 100, 120)[(i // 6) % 4]
    if fam == 0:
        rx, sm = rf"{tok} refused.{{0,{g}}}port \d+", f"{tok} refused by upstream 10.0.0.7 on port 8443"
    elif fam == 1:
        rx, sm = rf"pod .{{1,{g}}} in namespace {tok} .{{1,40}} failed", f"pod web-7f9c in namespace {tok} sync failed"
    elif fam == 2:
        rx, sm = rf"(?i)error.{{0,{g}}}{tok}.{{0,{g}}}retry", f"ERROR while calling {tok}, will retry in 5s"
    elif fam == 3:
        rx, sm = rf"(\w+\.){{2,}}{tok}Exception.{{0,{g}}}Caused by", f"com.acme.{tok}Exception: boom Caused by io"
    elif fam == 4:
        rx, sm = rf"{tok}.{{0,{g}}}(?:timed out|deadline exceeded)", f"{tok} call to db-0 deadline exceeded"
    else:
        rx, sm = rf"\b\d{{1,3}}(?:\.\d{{1,3}}){{3}}\b.{{0,{g}}}{tok} (?:refused|reset)", f"peer 10.1.2.3 said {tok} reset"
    srx, ssm = rf"{tok}Gap.{{0,{g // 2}}}code=\d+", f"{tok}Gap probe returned code=503"
    return rx, sm, srx, ssm


def _java_shape(rng: random.Random, tok: str, i: int) -> Tuple[str, str]:
    """The Java regex shapes a byte-DFA engine cannot hold, + a matching sample (planted after an
    ASCII noise prefix): wide bounded gaps (> 512 byte positions), Unicode properties, MULTILINE
    anchors inside a line (after U+2028), Unicode \\b, partial non-ASCII classes, UNICODE_CASE."""
    fam = i % 7
    if fam == 0:
        return rf"{tok} refused.{{0,600}}port \d+", f"{tok} refused by upstream 10.0.0.7 on port 8443"
    if fam == 1:
        return rf"(?i)error.{{0,300}}{tok}.{{0,300}}retry", f"ERROR while calling {tok} (état dégradé), will retry"
    if fam == 2:
        return rf"\p{{Lu}}\p{{L}}+{tok}Exception", f"caught Élan{tok}Exception in worker"
    if fam == 3:
        return rf"(?m)^\[{tok}\] (?:FATAL|ERROR)$", f"\u2028[{tok}] FATAL"
    if fam == 4:
        return rf"(?U)\b{tok}\w*Fehler\b", f"{tok}größeFehler erkannt"
    if fam == 5:
        return rf"[^\sé]+ {tok} échec", f"job-7 {tok} échec"
    return rf"(?iu){tok}: ÉCHEC .{{0,40}}Ä", f"{tok.upper()}: échec du contrôleur ä"


def make_library(n_patterns: int, seed: int = 0, n_sets: int = 4, secondary_rate: float = 0.7,
                 sequence_rate: float = 0.4, feature_mix: bool = True, short_literal_rate: float = 0.0,
                 literal_free_rate: float = 0.0, gap_rate: float = 0.0,
                 java_shape_rate: float = 0.0) -> Tuple[List[PatternSet], List[dict]]:
    """Returns (pattern sets, trigger descriptions used by ``make_log`` to plant matches).

    ``short_literal_rate`` / ``literal_free_rate`` / ``gap_rate`` / ``java_shape_rate``: shares of
    primaries whose only literal is a 3-6-byte code, that have no usable literal at all, that are
    bounded-gap regexes whose DFA blows up, or that use the Unicode / MULTILINE / wide-gap shapes of
    ``_java_shape`` (``realistic_library``)."""
    rng = random.Random(seed)
    sets = [{"metadata": {"library_id": f"synthetic-lib-{s}", "version": "1.0"}, "patterns": []}
            for s in range(n_sets)]
    triggers = []
    n_free = n_gap = n_java = 0
    for i in range(n_patterns):
        tok = _token(rng, i)
        style = rng.randrange(8) if feature_mix else 0
        u = rng.random()
        if u < literal_free_rate:
            style = 8
        elif u < literal_free_rate + short_literal_rate:
            style = 9
        elif u < literal_free_rate + short_literal_rate + gap_rate:
            style = 10
        elif u < literal_free_rate + short_literal_rate + gap_rate + java_shape_rate:
            style = 11
        gap_sec = None
        if style == 11:
            regex, sample = _java_shape(rng, tok, n_java)
            n_java += 1
        elif style == 10:
            regex, sample, srx, ssm = _bounded_gap(rng, tok, n_gap)
            gap_sec = (srx, ssm)
            n_gap += 1
        elif style == 8:
            regex, sample = _literal_free(rng, n_free)
            n_free += 1
        elif style == 9:
            code = _short_code(rng, 3 + i % 4)
            k = i % 3
            if k == 0:
                regex, sample = rf"\b{code}\b", f"fault {code} raised"
            elif k == 1:
                regex, sample = rf"(?i)\b{code}: \w+", f"{code.lower()}: aborted"
            else:
                regex, sample = rf"{code}\d*[a-z]?$", f"exit with {code}7"
        elif style == 0:
            regex, sample = tok + "Failure", f"{tok}Failure detected"
        elif style == 1:
            regex, sample = rf"(?i)\b{tok}\s+(crashed|aborted)\b", f"{tok.upper()} crashed unexpectedly"
        elif style == 2:
            regex, sample = rf"{tok}: code=\d{{3,5}}", f"{tok}: code={rng.randint(100, 99999)}"
        elif style == 3:
            regex, sample = rf"(Fatal|Severe) {tok} (state|status)", f"Fatal {tok} status reached"
        elif style == 4:
            regex, sample = rf"{tok}[A-Z]+Exception", f"caught {tok}PANICException in handler"
        elif style == 5:
            regex, sample = rf"^\[{tok}\] .*rejected", f"[{tok}] request was rejected"
        elif style == 6:
            regex, sample = rf"{tok}\.(conn|sock)[0-9]+ (lost|closed)$", f"{tok}.conn{rng.randint(0, 99)} lost"
        else:
            regex, sample = rf"{tok}-[a-f0-9]{{4}} timed? ?out", f"{tok}-{rng.randrange(16**4):04x} timed out"
        pat = {
            "id": f"pat-{i:05d}" if rng.random() > 0.02 else f"pat-{i // 2:05d}",
            "name": f"Synthetic failure {i}",
            "severity": rng.choice(SEVERITIES) if rng.random() > 0.03 else "weird",
            "primary_pattern": {"regex": regex, "confidence": round(rng.uniform(0.3, 0.95), 3)},
            "remediation": {"description": f"fix {tok}", "common_causes": ["synthetic"]},
        }
        secs, seqs, sec_samples = [], [], []
        if rng.random() < secondary_rate or gap_sec:
            for k in range(rng.randint(1, 3)):
                stok = f"{tok}Aux{k}"
                secs.append({"regex": stok if k else rf"(?i){stok}\b", "weight": round(rng.uniform(0.1, 0.9), 2),
                             "proximity_window": rng.choice([3, 5, 10, 20, 50, 200])})
                sec_samples.append(stok)
            if gap_sec:
                secs.append({"regex": gap_sec[0], "weight": 0.4, "proximity_window": 20})
                sec_samples.append(gap_sec[1])
            pat["secondary_patterns"] = secs
        if rng.random() < sequence_rate:
            evs = [{"regex": f"{tok}Step{k}"} for k in range(rng.randint(1, 3))]
            seqs.append({"description": f"{tok} lifecycle", "bonus_multiplier": round(rng.uniform(0.2, 1.5), 2),
                         "events": evs})
            pat["sequence_patterns"] = seqs
        if rng.random() < 0.8:
            pat["context_extraction"] = {"lines_before": rng.randint(0, 8), "lines_after": rng.randint(0, 6),
                                         "include_stack_trace": rng.random() < 0.5}
        sets[i % n_sets]["patterns"].append(pat)
        triggers.append({"sample": sample, "secondary": sec_samples,
                         "sequence": [e["regex"] for q in seqs for e in q["events"]]})
    return [PatternSet.model_validate(s) for s in sets], triggers


def backtracker_patterns(n: int, seed: int = 0) -> Tuple[PatternSet, List[dict]]:
    """``n`` primaries only a backtracker decides (backreferences, atomic groups /
    possessive quantifiers, lookarounds the automata do not express -- nested, or around a '$') +
    matching samples: n - 1 carry a pattern-specific literal (the device prefilter narrows them), the
    last one has none (its relaxed automaton runs in a literal-free scan group). The shapes real
    libraries use: a repeated id, "Fail" not followed by "ure", an error not preceded by "retrying",
    a restart loop of the same pod. (Plain lookaround clusters compile to DFAs: see
    ``lookaround_patterns``.)"""
    rng = random.Random(seed)
    pats, trig = [], []
    for i in range(n):
        tok = _token(rng, 10_000 + i)
        fam = i % 4
        if i == n - 1:
            rx, sm = r"^(\d{3})-(\d{4})-\2-\1$", "415-8812-8812-415"
        elif fam == 0:
            rx, sm = rf"(\w+) {tok}Loop \1\b", f"worker7 {tok}Loop worker7 again"
        elif fam == 1:
            rx, sm = rf"{tok}Fail(?!ure(?=\s))\w*", f"{tok}Failed to mount"
        elif fam == 2:
            rx, sm = rf"(?<!retrying )\b{tok}Err\b(?!.*done$)", f"fatal {tok}Err in worker"
        else:
            rx, sm = rf"(?i)(?>{tok}Lock)+\s+held", f"{tok.upper()}LOCK held by 7"
        pats.append({"id": f"bt-{i:04d}", "name": f"backtracker shape {i}", "severity": rng.choice(SEVERITIES),
                     "primary_pattern": {"regex": rx, "confidence": round(rng.uniform(0.3, 0.95), 3)}})
        trig.append({"sample": sm, "secondary": [], "sequence": []})
    ps = PatternSet.model_validate({"metadata": {"library_id": "backtracker", "version": "1.0"}, "patterns": pats})
    return ps, trig


def lookaround_patterns(n: int, seed: int = 0) -> Tuple[PatternSet, List[dict]]:
    """``n`` primaries with lookaround clusters used as line filters -- "Fail" not followed by "ure",
    an error not preceded by "retrying", ERROR with no "retry" later on the line, a token followed
    later by FATAL, an isolated word -- which compile to exact find() DFAs (jregex.cpp
    ``LookaroundDfa``), + matching samples."""
    rng = random.Random(seed)
    pats, trig = [], []
    for i in range(n):
        tok = _token(rng, 30_000 + i)
        fam = i % 5
        if fam == 0:
            rx, sm = rf"{tok}Fail(?!ure)\w*", f"{tok}Failed to mount"
        elif fam == 1:
            rx, sm = rf"(?<!retrying )\b{tok}Err\b", f"fatal {tok}Err in worker"
        elif fam == 2:
            rx, sm = rf"\b{tok}ERROR\b(?!.*retry)", f"{tok}ERROR disk full"
        elif fam == 3:
            rx, sm = rf"(?=.*FATAL){tok}Err", f"{tok}Err then FATAL"
        else:
            rx, sm = rf"(?<!\S){tok}x(?!\S)", f"got {tok}x here"
        pats.append({"id": f"la-{i:04d}", "name": f"lookaround shape {i}", "severity": rng.choice(SEVERITIES),
                     "primary_pattern": {"regex": rx, "confidence": round(rng.uniform(0.3, 0.95), 3)}})
        trig.append({"sample": sm, "secondary": [], "sequence": []})
    ps = PatternSet.model_validate({"metadata": {"library_id": "lookaround", "version": "1.0"}, "patterns": pats})
    return ps, trig


def counted_repeat_patterns(n: int, seed: int = 0) -> Tuple[PatternSet, List[dict]]:
    """``n`` primaries with a wide bounded repeat of one class (``X.{0,2100}Y``,
    ``X[^;]{0,5000}Y``, ``X\\S{0,20000}Y``): the regular shapes past the 2,048-position BPG limit
    that compile to a counted position (csrc/regex/jregex.cpp ``Glushkov`` counters) + matching
    samples."""
    rng = random.Random(seed)
    pats, trig = [], []
    shapes = ((r"{a}.{{0,2100}}{b}", "{a} then some text {b}"),
              (r"{a}[^;]{{0,5000}}{b}", "{a} waited {b}"),
              (r"{a}\S{{0,20000}}{b}", "{a}/x/y/{b}"))
    for i in range(n):
        a, b = _token(rng, 20_000 + 2 * i), _token(rng, 20_001 + 2 * i)
        rx, sm = shapes[i % len(shapes)]
        pats.append({"id": f"cr-{i:04d}", "name": f"counted repeat {i}", "severity": rng.choice(SEVERITIES),
                     "primary_pattern": {"regex": rx.format(a=a, b=b), "confidence": round(rng.uniform(0.3, 0.95), 3)}})
        trig.append({"sample": sm.format(a=a, b=b), "secondary": [], "sequence": []})
    ps = PatternSet.model_validate({"metadata": {"library_id": "counted", "version": "1.0"}, "patterns": pats})
    return ps, trig


def realistic_library(n_patterns: int, seed: int = 0, **kw):
    """The headline bench library: the synthetic mix plus ~10% primaries with only a 3-6-byte
    literal, ~5% literal-free primaries, ~1.5% bounded-gap primaries (``X.{0,120}Y``, each
    with a bounded-gap secondary) and ~1% Unicode / MULTILINE / wide-gap shapes
    (``X.{0,600}Y``, ``\\p{L}``, ``(?m)^..$``, ``(?U)\\b``, ``[^é]``, ``(?iu)``) -- the shapes real
    libraries have (short error codes, IP:port, `^\\s+at ...` stack frames, "refused ... port N")
    and the matcher's worst cases."""
    kw.setdefault("short_literal_rate", 0.10)
    kw.setdefault("literal_free_rate", 0.05)
    kw.setdefault("gap_rate", 0.015)
    kw.setdefault("java_shape_rate", 0.01)
    return make_library(n_patterns, seed=seed, **kw)


def _noise_line(rng: random.Random, i: int) -> str:
    lvl = rng.choice(LEVELS)
    comp = rng.choice(COMPONENTS)
    msg = " ".join(rng.choice(WORDS) for _ in range(rng.randint(4, 12)))
    return f"2025-09-19T12:{(i // 60) % 60:02d}:{i % 60:02d}.{i % 1000:03d}Z {lvl:5s} [{comp}] {msg} id={rng.randint(0, 1 << 30)}"


def make_log(n_lines: int, triggers: List[dict], seed: int = 0, hit_rate: float = 0.01,
             aux_rate: float = 0.01, stack_rate: float = 0.01, crlf_rate: float = 0.0) -> str:
    rng = random.Random(seed)
    out = []
    i = 0
    while i < n_lines:
        r = rng.random()
        if triggers and r < hit_rate:
            t = rng.choice(triggers)
            if t["sequence"] and rng.random() < 0.6:
                for ev in t["sequence"][:-1]:
                    out.append(f"INFO [app] {ev} reached")
                    i += 1
            if t["sample"][:1].isspace():          # anchored stack-frame shape: a line of its own
                out.append(t["sample"])
            else:
                out.append(_noise_line(rng, i)[:40] + " " + t["sample"])
            if t["sequence"] and rng.random() < 0.6:
                out.append(f"INFO [app] {t['sequence'][-1]} reached")
                i += 1
            if t["secondary"] and rng.random() < 0.7:
                out.append(f"WARN [app] saw {rng.choice(t['secondary'])} nearby")
                i += 1
        elif triggers and r < hit_rate + aux_rate:
            t = rng.choice(triggers)
            if t["secondary"]:
                out.append(f"DEBUG [app] {rng.choice(t['secondary'])} event")
            else:
                out.append(_noise_line(rng, i))
        elif r < hit_rate + aux_rate + stack_rate:
            out.append(f"ERROR [app] {rng.choice(EXC)}: boom")
            for k in range(rng.randint(1, 6)):
                out.append(f"\tat com.example.svc{k}.Handler$Inner.run(Handler.java:{rng.randint(1, 999)})")
                i += 1
        else:
            out.append(_noise_line(rng, i))
        i += 1
    sep = "\n"
    if crlf_rate > 0:
        parts = []
        for line in out:
            parts.append(line)
            parts.append("\r\n" if rng.random() < crlf_rate else "\n")
        return "".join(parts)
    return sep.join(out) + sep
