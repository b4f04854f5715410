"""C++ Java-regex compiler (DFA path) vs the independent javacompat oracle; literal soundness."""
import random

import pytest
from hypothesis import given, settings, HealthCheck
from hypothesis import strategies as st

from log_parser_amd.native import N
from log_parser_amd.regex.javacompat import java_find

CORPUS = [
    r"OutOfMemoryError", r"(?i)\b(ERROR|FATAL|CRITICAL|SEVERE)\b", r"(?i)\b(WARN|WARNING)\b",
    r"^\s*at\s+[\w\.\$]+\(.*\)\s*$", r"\b\w*Exception\b|\b\w*Error\b", r"Connection (refused|reset)",
    r"colou?r", r"\d{3,}ms", r"abc$", r"^$", r"x*", r"[^a]b", r"\bfoo", r"a.c", r"(?i)warn(ing)?",
    r"Back-off restarting failed container", r"OOMKilled|exit code 137", r"panic: .*",
    r"(?i)connection (timed out|refused)", r"\[(ERROR|FATAL)\]", r"\QA.B\E", r"[a-c[x-z]]+", r"\x41B\t",
    r"ab{2,3}c", r"(ab|a)(bc|c)", r"^(?:(?i)err)or", r"\B-\B", r"\p{Upper}{2}\p{Digit}", r"[\w&&[^\d]]+9",
    r"a\Z", r"a\z", r"\Aab", r"(a|b)*abb", r"é+x", r"[^\s]+@[^\s]+", r"time(d)? ?out", r"\\n",
    r"(?x) a b # comment", r"(?s)a.b", r"\h+x", r"x{0}y", r"(?i)stra[sß]e",
]
LINES = [
    "java.lang.OutOfMemoryError: heap", "ERROR: x", "  at com.foo.Bar(Bar.java:12)", "  at com.foo.Bar(Bar.java:12) x",
    "NullPointerException", "MyError", "xError1", "Connection refused", "color", "colour", "took 1234ms",
    "took 12ms", "abc", "abc\r", "abcd", "", "éb", "ab", "foo", "xfoo", "a\rc", "aéc", "WARNING", "warnings",
    "Back-off restarting failed container x", "exit code 137", "panic: oops", "CONNECTION TIMED OUT",
    "[FATAL] boom", "A.B", "AxB", "yyy", "AB\t", "abbc", "abbbbc", "abc", "error", "ERROR", "a-b", " - ",
    "AB1", "ab9", "a\r", "a", "ab", "aabb", "ééx", "x@y", "timed out", "timeout", "\\n", "ab", "a\nb",
    "   x", "y", "STRASSE", "straße",
]


@pytest.mark.parametrize("pat", CORPUS)
def test_corpus_dfa_matches_oracle(pat):
    d = N.compile_regex(pat)
    if d["kind"] != 0:
        pytest.skip(f"not a DFA regex ({d['error']})")
    for line in LINES:
        try:
            want = java_find(pat, line)
        except Exception:
            pytest.skip("oracle cannot translate")
        got = N.dfa_find(pat, line.encode())
        assert got == want, (pat, line)
        if got and d["has_literals"]:
            low = line.encode().lower()
            assert any(l in low for l in d["literals"]), (pat, line, d["literals"])


def test_unsupported_and_invalid_are_classified():
    assert N.compile_regex(r"(a)\1")["kind"] == 2          # backreference -> host fallback
    assert N.compile_regex(r"foo(?=bar)")["kind"] == 0     # lookaround cluster -> exact find() DFA
    assert N.compile_regex(r"a(?=b(?!c))")["kind"] == 2    # nested lookaround -> host fallback
    assert N.compile_regex(r"a(?!.*x$)")["kind"] == 2      # '$' inside a lookaround -> host fallback
    assert N.compile_regex(r"a*+b")["kind"] == 2           # possessive -> host fallback
    assert N.compile_regex(r"(abc")["kind"] == 3           # syntax error
    assert N.compile_regex(r"a**")["kind"] == 3
    assert N.compile_regex(r"{")["kind"] == 3              # Java: Illegal repetition
    big = N.compile_regex(r"(a|b)*a(a|b){14}", max_states=512)
    assert big["kind"] == 1                                 # DFA blow-up -> NFA path


# ---- randomized differential testing over a regex grammar ---------------------------------
ATOMS = ["a", "b", "c", "A", "B", " ", "1", "-", ".", r"\d", r"\w", r"\s", r"\W", "[ab]", "[^a]", "[a-c]",
         r"\.", "é", r"\b", r"\B", "^", "$"]


def _rand_regex(rng: random.Random, depth=0) -> str:
    n = rng.randint(1, 4)
    parts = []
    for _ in range(n):
        r = rng.random()
        if r < 0.15 and depth < 2:
            inner = "|".join(_rand_regex(rng, depth + 1) for _ in range(rng.randint(1, 3)))
            a = "(" + inner + ")"
        else:
            a = rng.choice(ATOMS)
        if a not in ("^", "$", r"\b", r"\B"):
            q = rng.random()
            if q < 0.15:
                a += "*"
            elif q < 0.25:
                a += "+"
            elif q < 0.35:
                a += "?"
            elif q < 0.4:
                lo = rng.randint(0, 2)
                a += "{%d,%d}" % (lo, lo + rng.randint(0, 2))
        parts.append(a)
    s = "".join(parts)
    if rng.random() < 0.15:
        s = "(?i)" + s
    return s


def _rand_line(rng: random.Random) -> str:
    alpha = "abcAB 1-.é_\t"
    s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 12)))
    if rng.random() < 0.1:
        s += "\r"
    return s


@settings(max_examples=300, deadline=None, suppress_health_check=list(HealthCheck))
@given(st.integers(min_value=0, max_value=2**31 - 1))
def test_random_regexes_match_oracle(seed):
    rng = random.Random(seed)
    pat = _rand_regex(rng)
    d = N.compile_regex(pat)
    if d["kind"] != 0:
        return
    for _ in range(25):
        line = _rand_line(rng)
        try:
            want = java_find(pat, line)
        except Exception:
            return
        got = N.dfa_find(pat, line.encode())
        assert got == want, (pat, line)
        if got and d["has_literals"]:
            low = line.encode().lower()
            assert any(l in low for l in d["literals"]), (pat, line, d["literals"])
