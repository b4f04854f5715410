"""java.util.regex -> Python ``regex`` translation (oracle + host fallback only).

Used by the pure-Python golden model (``golden.py``) and as the *host fallback* for the few
non-regular constructs the automaton engine refuses (backreferences, lookaround, possessive /
atomic groups). It is intentionally independent of the C++ regex compiler so that the golden
oracle does not share a parser with the GPU engine.

Java 21 defaults reproduced: ``\\w \\d \\s \\b`` and CASE_INSENSITIVE are ASCII-only;
``.`` excludes ``\\n \\r \\u0085 \\u2028 \\u2029``; without MULTILINE ``$`` / ``\\Z`` match at the end
of input or before a final line terminator; ``\\z`` is the absolute end; ``\\h``/``\\v``/``\\R`` are
Java's horizontal/vertical whitespace and linebreak; POSIX ``\\p{..}`` classes are ASCII.
"""
from __future__ import annotations

import functools

import regex as _re

_TERM = "\\r\\x85\u2028\u2029"
DOT = "[^\\n" + _TERM + "]"
DOT_UNIX = r"[^\n]"
EOL = r"(?=(?:\r\n|[\n" + _TERM + r"])?\Z)"
EOL_UNIX = r"(?=\n?\Z)"
EOL_MULTI = r"(?=[\n" + _TERM + r"]|\Z)"
BOL_MULTI = r"(?:\A|(?<=[\n" + _TERM + r"])(?!\Z))"

_H = " \\t\xa0\u1680\u180e\u2000-\u200a\u202f\u205f\u3000"
_V = "\\n\\x0b\\f\\r\x85\u2028\u2029"

_POSIX = {
    "Lower": "a-z", "Upper": "A-Z", "ASCII": r"\x00-\x7f", "Alpha": "a-zA-Z", "Digit": "0-9",
    "Alnum": "a-zA-Z0-9", "Punct": r"!-/:-@\[-`{-~", "Graph": r"!-~", "Print": r" -~",
    "Blank": r" \t", "Cntrl": r"\x00-\x1f\x7f", "XDigit": "0-9a-fA-F", "Space": r" \t\n\x0b\f\r",
    "javaLowerCase": "a-z", "javaUpperCase": "A-Z", "javaWhitespace": r" \t\n\x0b\f\r\x1c-\x1f",
}


class UnsupportedJavaRegex(ValueError):
    pass


def _class_body_for_escape(esc: str, neg: bool):
    """Return (body, negated) for a class-like escape usable inside [...]."""
    m = {"d": ("0-9", False), "D": ("0-9", True), "s": (r" \t\n\x0b\f\r", False),
         "S": (r" \t\n\x0b\f\r", True), "w": ("a-zA-Z0-9_", False), "W": ("a-zA-Z0-9_", True),
         "h": (_H, False), "H": (_H, True), "v": (_V, False), "V": (_V, True)}
    return m[esc]


def _char_escape(p: str, i: int):
    """Parse a Java single-char escape at p[i] (after the backslash). Returns (python_text, new_i)
    or None if not a single-char escape."""
    c = p[i]
    simple = {"t": "\\t", "n": "\\n", "r": "\\r", "f": "\\f", "a": "\\x07", "e": "\\x1b"}
    if c in simple:
        return simple[c], i + 1
    if c == "0":
        j = i + 1
        digs = ""
        while j < len(p) and len(digs) < 3 and p[j] in "01234567":
            digs += p[j]
            j += 1
        if not digs:
            raise UnsupportedJavaRegex("illegal octal escape")
        v = int(digs, 8)
        if v > 0o377:
            digs = digs[:-1]
            j -= 1
            v = int(digs, 8)
        return "\\x%02x" % v, j
    if c == "x":
        if i + 1 < len(p) and p[i + 1] == "{":
            j = p.index("}", i + 2)
            return _re.escape(chr(int(p[i + 2:j], 16))), j + 1
        return _re.escape(chr(int(p[i + 1:i + 3], 16))), i + 3
    if c == "u":
        return _re.escape(chr(int(p[i + 1:i + 5], 16))), i + 5
    if c == "c":
        return _re.escape(chr(ord(p[i + 1]) ^ 64)), i + 2
    if not c.isalnum():
        return _re.escape(c), i + 1
    return None


def _posix(p: str, i: int):
    """p[i] is 'p' or 'P'. Returns (body, negated, new_i) for a bracket-able class."""
    neg = p[i] == "P"
    if p[i + 1] == "{":
        j = p.index("}", i + 2)
        name = p[i + 2:j]
        ni = j + 1
    else:
        name = p[i + 1]
        ni = i + 2
    if name.startswith("^"):
        neg = not neg
        name = name[1:]
    key = name[2:] if name.startswith("Is") and name[2:] in _POSIX else name
    if key in _POSIX:
        return _POSIX[key], neg, ni
    # unicode property: let the regex module interpret it
    return None, (("\\P{%s}" if neg else "\\p{%s}") % name), ni


@functools.lru_cache(maxsize=65536)
def to_python(pattern: str) -> str:
    p = pattern
    out = []
    # scope stack: dict(dotall, multiline, unix, comments, pending_closes)
    scopes = [dict(s=False, m=False, d=False, x=False, close=0)]
    i = 0
    n = len(p)

    def cur():
        return scopes[-1]

    def parse_flags(j):
        on, off, neg = "", "", False
        while j < n and p[j] not in "):":
            ch = p[j]
            if ch == "-":
                neg = True
            elif ch in "idmsuxU":
                if neg:
                    off += ch
                else:
                    on += ch
            else:
                raise UnsupportedJavaRegex("bad inline flag %r" % ch)
            j += 1
        return on, off, j

    def apply(scope, on, off):
        s = dict(scope)
        for ch, v in [(c, True) for c in on] + [(c, False) for c in off]:
            if ch in "smdx":
                s[ch] = v
            elif ch == "U":
                raise UnsupportedJavaRegex("UNICODE_CHARACTER_CLASS")
        return s

    def ci_prefix(on, off):
        on_i = "i" in on
        off_i = "i" in off
        if on_i:
            return "(?i:"
        if off_i:
            return "(?-i:"
        return None

    while i < n:
        c = p[i]
        sc = cur()
        if sc["x"] and c in " \t\n\r\f\x0b":
            i += 1
            continue
        if sc["x"] and c == "#":
            while i < n and p[i] != "\n":
                i += 1
            continue
        if c == "\\":
            i += 1
            if i >= n:
                raise UnsupportedJavaRegex("trailing backslash")
            e = p[i]
            if e == "Q":
                j = p.find("\\E", i + 1)
                lit = p[i + 1:] if j < 0 else p[i + 1:j]
                out.append(_re.escape(lit))
                i = n if j < 0 else j + 2
                continue
            if e in "dDsSwWhHvV":
                body, neg = _class_body_for_escape(e, False)
                out.append(("[^%s]" if neg else "[%s]") % body)
                i += 1
                continue
            if e in "pP":
                body, neg, i = _posix(p, i)
                if body is None:
                    out.append(neg)
                else:
                    out.append(("[^%s]" if neg else "[%s]") % body)
                continue
            if e == "b":
                out.append("\\b")
                i += 1
                continue
            if e == "B":
                out.append("\\B")
                i += 1
                continue
            if e == "A":
                out.append("\\A")
                i += 1
                continue
            if e == "z":
                out.append("\\Z")
                i += 1
                continue
            if e == "Z":
                out.append(EOL_UNIX if sc["d"] else EOL)
                i += 1
                continue
            if e == "G":
                out.append("\\G")
                i += 1
                continue
            if e == "R":
                out.append("(?:\\r\\n|[" + _V + "])")
                i += 1
                continue
            if e == "X":
                out.append("\\X")
                i += 1
                continue
            if e == "k":
                j = p.index(">", i)
                out.append("(?P=%s)" % p[i + 2:j])
                i = j + 1
                continue
            if e.isdigit() and e != "0":
                j = i
                while j < n and p[j].isdigit():
                    j += 1
                out.append("\\" + p[i:j])
                i = j
                continue
            r = _char_escape(p, i)
            if r is None:
                raise UnsupportedJavaRegex("unknown escape \\%s" % e)
            out.append(r[0])
            i = r[1]
            continue
        if c == "[":
            body, i = _parse_class(p, i)
            out.append(body)
            continue
        if c == ".":
            out.append("(?s:.)") if sc["s"] else out.append(DOT_UNIX if sc["d"] else DOT)
            i += 1
            continue
        if c == "$":
            if sc["m"]:
                out.append(EOL_MULTI)
            else:
                out.append(EOL_UNIX if sc["d"] else EOL)
            i += 1
            continue
        if c == "^":
            out.append(BOL_MULTI if sc["m"] else "\\A")
            i += 1
            continue
        if c == "(":
            if p.startswith("(?", i):
                k = i + 2
                if k < n and p[k] in "=!>" or p.startswith("<=", k) or p.startswith("<!", k):
                    # lookaround / atomic: pass through
                    tok = "(?" + (p[k:k + 2] if p[k] == "<" else p[k])
                    out.append(tok)
                    i = k + (2 if p[k] == "<" else 1)
                    scopes.append(dict(sc, close=0))
                    continue
                if k < n and p[k] == "<":
                    j = p.index(">", k)
                    out.append("(?P<%s>" % p[k + 1:j])
                    i = j + 1
                    scopes.append(dict(sc, close=0))
                    continue
                on, off, j = parse_flags(k)
                if j < n and p[j] == ")":
                    # (?flags) : applies until end of the enclosing group
                    nsc = apply(sc, on, off)
                    pre = ci_prefix(on, off)
                    if pre:
                        out.append(pre)
                        nsc["close"] = sc["close"] + 1
                        nsc.setdefault("reopen", [])
                        nsc["reopen"] = list(sc.get("reopen", [])) + [pre]
                    scopes[-1] = nsc
                    i = j + 1
                    continue
                if j < n and p[j] == ":":
                    pre = ci_prefix(on, off) or "(?:"
                    out.append(pre)
                    scopes.append(dict(apply(sc, on, off), close=0, reopen=[]))
                    i = j + 1
                    continue
                raise UnsupportedJavaRegex("bad group")
            out.append("(")
            scopes.append(dict(sc, close=0, reopen=[]))
            i += 1
            continue
        if c == ")":
            out.append(")" * sc["close"])
            if len(scopes) > 1:
                scopes.pop()
            out.append(")")
            i += 1
            continue
        if c == "|":
            out.append(")" * sc["close"])
            out.append("|")
            out.extend(sc.get("reopen", []))
            i += 1
            continue
        if c == "{":
            # Java: '{' must start a valid repetition
            j = p.find("}", i)
            if j < 0 or not _re.fullmatch(r"\d+(,\d*)?", p[i + 1:j]):
                raise UnsupportedJavaRegex("Illegal repetition")
            out.append(p[i:j + 1])
            i = j + 1
            continue
        out.append(_re.escape(c) if c not in "*+?" else c)
        i += 1
    out.append(")" * cur()["close"])
    return "".join(out)


def _parse_class(p: str, i: int):
    """Parse a Java character class starting at p[i]=='['; supports nested unions (flattened)."""
    assert p[i] == "["
    i += 1
    neg = False
    if i < len(p) and p[i] == "^":
        neg = True
        i += 1
    parts = []
    first = True
    while True:
        if i >= len(p):
            raise UnsupportedJavaRegex("Unclosed character class")
        c = p[i]
        if c == "]" and not first:
            i += 1
            break
        first = False
        if c == "[":
            sub, i = _parse_class(p, i)
            if sub.startswith("[^"):
                raise UnsupportedJavaRegex("negated nested class")
            parts.append(sub[1:-1])
            continue
        if c == "&" and p.startswith("&&", i):
            raise UnsupportedJavaRegex("class intersection")
        if c == "\\":
            e = p[i + 1]
            if e == "Q":
                j = p.find("\\E", i + 2)
                lit = p[i + 2:j]
                parts.append("".join(_cls_escape(ch) for ch in lit))
                i = j + 2
                continue
            if e in "dDsSwWhHvV":
                body, ng = _class_body_for_escape(e, False)
                if ng:
                    if len(parts) == 0 and p[i + 2] == "]" and not neg:
                        # [\D] alone
                        return "[^%s]" % body, i + 3
                    raise UnsupportedJavaRegex("negated escape inside class")
                parts.append(body)
                i += 2
                continue
            if e in "pP":
                body, ng, ni = _posix(p, i + 1)
                if body is None or ng:
                    raise UnsupportedJavaRegex("unicode/negated property in class")
                parts.append(body)
                i = ni
                continue
            r = _char_escape(p, i + 1)
            if r is None:
                raise UnsupportedJavaRegex("bad class escape")
            parts.append(r[0] if r[0].startswith("\\") else _cls_escape(r[0].replace("\\", "")))
            i = r[1]
            continue
        if c == "-" and parts and i + 1 < len(p) and p[i + 1] not in "]":
            parts.append("-")
            i += 1
            continue
        parts.append(_cls_escape(c))
        i += 1
    body = "".join(parts)
    return ("[^%s]" if neg else "[%s]") % body, i


def _cls_escape(ch: str) -> str:
    if ch in "\\]^-[":
        return "\\" + ch
    return ch


@functools.lru_cache(maxsize=65536)
def compile_java(pattern: str):
    """Compile a Java regex into a Python ``regex`` object with Java-equivalent semantics."""
    return _re.compile(to_python(pattern), _re.ASCII | _re.V0)


def java_find(pattern: str, line: str) -> bool:
    return compile_java(pattern).search(line) is not None
