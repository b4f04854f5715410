"""Correctness anchors from SURVEY §6.2 / BASELINE.md (the reference's code, not its doc errata)."""
import math

from log_parser_amd import golden
from log_parser_amd.frequency import FrequencyState
from log_parser_amd.utils.config import ScoringParams

P = ScoringParams()


def test_chronological_anchors():
    assert golden.chronological_factor(0, 100, P) == 2.5
    assert math.isclose(golden.chronological_factor(20, 100, P), 1.5)
    assert math.isclose(golden.chronological_factor(50, 100, P), 1.0)
    assert math.isclose(golden.chronological_factor(15, 100, P), 1.75)   # doc says ~2.1 (erratum)
    assert math.isclose(golden.chronological_factor(99, 100, P), 0.51)


def test_proximity_anchor():
    assert math.isclose(1.0 + 0.8 * math.exp(-5 / 10.0), 1.48522, rel_tol=1e-5)


def test_worked_example_code_consistent():
    # 0.8 x 3.0 x chrono 1.75 x prox 1.4445 x 1.0 x ctx 2.0 = 12.1337 (doc's 21.17 is an arithmetic error)
    assert math.isclose(0.8 * 3.0 * 1.75 * 1.4445 * 1.0 * 2.0, 12.1338, rel_tol=1e-4)
    assert math.isclose(0.8 * 3.0 * 2.1 * 1.4 * 1.0 * 1.5, 10.584, rel_tol=1e-9)


def test_context_factor_two_errors_one_stack():
    lines = ["ERROR one", "ERROR two", "    at com.x.Y.z(Y.java:1)"]
    # 1 + 0.4 + 0.4 + 0.1 + min(0.1, 0.5) = 2.0 (doc says ~1.5)
    assert math.isclose(golden.context_factor(lines, P), 2.0)


def test_frequency_penalty_schedule():
    t = [1000.0]
    tr = golden.FrequencyTracker(P, clock=lambda: t[0])
    pens = []
    for _ in range(25):
        pens.append(tr.penalty("x"))
        tr.record("x")
    assert pens[:11] == [0.0] * 11
    for k in range(11, 25):
        assert math.isclose(pens[k], min(0.8, (k - 10) / 10.0))
    t[0] += 3601
    assert tr.penalty("x") == 0.0      # slid out of the 1 h window


def test_split_lines_java_semantics():
    assert golden.split_lines("") == [""]
    assert golden.split_lines("\n") == []
    assert golden.split_lines("\n\n\r\n") == []
    assert golden.split_lines("a\r\nb\n\nc\n\n") == ["a", "b", "", "c"]
    assert golden.split_lines("a\rb") == ["a\rb"]
    assert golden.split_lines("\na") == ["", "a"]
    assert golden.split_lines("a\r\r\n") == ["a\r"]


def test_summary_rules():
    mk = lambda s: {"matchedPattern": {"severity": s}}  # noqa: E731
    assert golden.build_summary([])["highestSeverity"] == "NONE"
    s = golden.build_summary([mk("low"), mk("HIGH"), mk("weird")])
    assert s["highestSeverity"] == "HIGH" and s["severityDistribution"] == {"LOW": 1, "HIGH": 1, "WEIRD": 1}
    assert golden.build_summary([mk("b"), mk("a")])["highestSeverity"] == "B"


def test_frequency_state_snapshot(tmp_path):
    t = [0.0]
    st = FrequencyState(1, clock=lambda: t[0])
    st.record_counts(["a", "b"], [3, 0])
    st.record_counts(["a"], [2])
    assert list(st.carry(["a", "b", "c"])) == [5, 0, 0]
    p = str(tmp_path / "f.json")
    st.snapshot(p)
    st2 = FrequencyState(1, clock=lambda: t[0])
    st2.restore(p)
    assert list(st2.carry(["a"])) == [5]
    t[0] = 3600.5
    assert list(st2.carry(["a"])) == [0]
    assert st.get_pattern_frequency("zzz") is None


def test_pack_split_docs_equals_java_split():
    """Native batch staging (csrc/io/docs.cpp) == Java String.split per document, for str and
    bytes bodies, across the parallel document partition."""
    import random
    import numpy as np
    from log_parser_amd.native import N
    from log_parser_amd import golden
    rng = random.Random(3)
    docs = ["", "\n", "\n\n", "a", "a\n", "a\r\n\r\n", "\r\n", "x\ry\n", "é\nü\r\n"]
    for _ in range(400):
        parts = [rng.choice(["", "a", "\r", "é", "line with words", "日本"]) * rng.randint(0, 4) +
                 rng.choice(["\n", "\r\n", "\n", ""]) for _ in range(rng.randint(0, 60))]
        docs.append("".join(parts))
    docs += ["z" * 300000 + "\n" + "y" * 10] * 12          # > 1 MiB total: several threads
    total = sum(len(d.encode()) for d in docs)
    buf = np.zeros(total + 64, np.uint8)
    for nthreads in (1, 8):
        ls, ll, dl, off = N.pack_split_docs(docs, buf.ctypes.data, buf.size, nthreads)
        blob = buf[:total].tobytes()
        assert blob == "".join(docs).encode()
        for d, s in enumerate(docs):
            got = [blob[a:a + b].decode() for a, b in zip(ls[dl[d]:dl[d + 1]], ll[dl[d]:dl[d + 1]])]
            assert got == golden.split_lines(s), (d, s[:40])
    assert N.pack_split_docs(docs, buf.ctypes.data, 10, 1) == total       # too small: needed size
    assert N.pack_split_docs(["a\ud800b"], buf.ctypes.data, buf.size, 1) is None   # lone surrogate


def test_blank_pattern_ids_follow_java_trim():
    """FrequencyTrackingService.java:42,65 -- ``id.trim().isEmpty()``: Java trims every char <=
    U+0020 and nothing else. Ids made of control chars are blank (never penalised); a non-breaking
    or em space is a real id (penalised past the threshold), unlike Python's str.strip()."""
    import torch
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.models.schema import PatternSet
    from log_parser_amd.utils.config import Config
    assert golden.java_blank(None) and golden.java_blank("") and golden.java_blank(" \t\x01\x1f")
    assert not golden.java_blank("\u00a0") and not golden.java_blank("\u2003") and not golden.java_blank(" a ")
    ids = ["\x01", "\u00a0", "\u2003 ", " \x0b "]
    pats = [{"id": pid, "name": f"p{i}", "severity": "HIGH",
             "primary_pattern": {"regex": f"tok{i}x", "confidence": 0.5}} for i, pid in enumerate(ids)]
    sets = [PatternSet.model_validate({"metadata": {"library_id": "ids"}, "patterns": pats})]
    logs = "\n".join(f"line tok{k % 4}x here" for k in range(100))
    p = ScoringParams()
    lib = CompiledLibrary(sets, p)
    assert lib.freq_ids == ["\u00a0", "\u2003 "]
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    r = eng.analyze(logs)
    g = golden.analyze(logs, sets, p, golden.FrequencyTracker(p))
    assert [e["score"] for e in r["events"]] == [e["score"] for e in g["events"]]
    last = {e["matchedPattern"]["name"]: e["score"] for e in g["events"]}
    assert last["p1"] < last["p0"]           # U+00A0 id: 25 matches > threshold -> penalised
