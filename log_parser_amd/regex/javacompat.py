"""java.util.regex -> Python ``regex`` translation: the TEST ORACLE.

Used by the pure-Python golden model (``golden.py``) and by the regex tests as the independent
reference for Java's ``find()``. The engine never runs it: regular regexes run on the automata
(DFA / BPG programs) and the non-regular ones (backreferences, lookaround, possessive / atomic
groups) on the native C++ backtracker (``jregex.cpp BtRegex``). It is intentionally independent of
the C++ regex compiler so that the oracle does not share a parser with the engine.

Java 21 defaults reproduced: ``\\w \\d \\s \\b`` and CASE_INSENSITIVE are ASCII-only;
``.`` excludes ``\\n \\r \\u0085 \\u2028 \\u2029``; without MULTILINE ``$`` / ``\\Z`` match at the end
of input or before a final line terminator; ``\\z`` is the absolute end; ``\\h``/``\\v``/``\\R`` are
Java's horizontal/vertical whitespace and linebreak; POSIX ``\\p{..}`` classes are ASCII.

Character classes are evaluated here as explicit code-point range sets (nesting, negation,
``&&`` intersection, predefined and property escapes, CASE_INSENSITIVE closure) and emitted as
ranges; ``\\p{..}`` names are resolved with Java's rules (``In`` block / ``Is`` property, category
or script / ``name=value`` / POSIX, CharPredicates) against the generated Unicode tables
(``N.unicode_set``); ``(?U)`` switches ``\\w \\d \\s \\b`` and POSIX classes to Unicode and, with
``(?iu)``, case-insensitive literals and ranges use Java's simple upper / lower case mappings
(``Character.toUpperCase`` / ``toLowerCase``, built here from Python's ``str.upper`` / ``lower``).
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


# ---- explicit code-point sets (sorted disjoint ranges) --------------------------------------
MAXCP = 0x10FFFF


def _norm(rs):
    out = []
    for lo, hi in sorted(rs):
        if out and lo <= out[-1][1] + 1:
            if hi > out[-1][1]:
                out[-1] = (out[-1][0], hi)
        else:
            out.append((lo, hi))
    return out


def _neg(rs):
    out, nxt = [], 0
    for lo, hi in rs:
        if lo > nxt:
            out.append((nxt, lo - 1))
        nxt = hi + 1
    if nxt <= MAXCP:
        out.append((nxt, MAXCP))
    return out


def _inter(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if lo <= hi:
            out.append((lo, hi))
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def _chr(c: int) -> str:
    return "\\U%08x" % c


def _emit(rs, neg=False) -> str:
    if neg:
        rs = _neg(_norm(rs))
    rs = _norm(rs)
    if not rs:
        return "(?!)"
    return "[" + "".join(_chr(lo) if lo == hi else _chr(lo) + "-" + _chr(hi) for lo, hi in rs) + "]"


@functools.lru_cache(maxsize=None)
def _uset(key: str):
    from ..native import N
    return tuple((int(a), int(b)) for a, b in N.unicode_set(key))


@functools.lru_cache(maxsize=1)
def _case_pairs():
    """(c, upper(c)) and (c, lower(c)) pairs of Java's simple case mappings (single code point)."""
    up, lo = {}, {}
    for c in range(MAXCP + 1):
        if 0xD800 <= c <= 0xDFFF:
            continue
        ch = chr(c)
        u, w = ch.upper(), ch.lower()
        if len(u) == 1 and u != ch:
            up[c] = ord(u)
        if len(w) == 1 and w != ch:
            lo[c] = ord(w)
    adj = {}
    for m in (up, lo):
        for a, b in m.items():
            adj.setdefault(a, set()).add(b)
            adj.setdefault(b, set()).add(a)
    return up, lo, adj


def _case_variants(c: int, unicode_case: bool):
    """Code points equal to c under Java CASE_INSENSITIVE (ASCII) / + UNICODE_CASE (SingleU)."""
    if not unicode_case:
        if 97 <= c <= 122:
            return [c, c - 32]
        if 65 <= c <= 90:
            return [c, c + 32]
        return [c]
    up, lo, adj = _case_pairs()
    key = lambda x: lo.get(up.get(x, x), up.get(x, x))  # noqa: E731
    seen, todo, out = {c}, [c], []
    while todo:
        x = todo.pop()
        if key(x) == key(c):
            out.append(x)
        for y in adj.get(x, ()):
            if y not in seen:
                seen.add(y)
                todo.append(y)
    return out


def _ci_range(lo: int, hi: int, unicode_case: bool):
    """Java CIRange / CIRangeU: ch matches when its (ASCII / simple) upper or lower case is in range."""
    rs = [(lo, hi)]
    if not unicode_case:
        for c in range(65, 91):
            if lo <= c + 32 <= hi:
                rs.append((c, c))
            if lo <= c <= hi:
                rs.append((c + 32, c + 32))
        return rs
    up, low, _ = _case_pairs()
    for m in (up, low):
        for a, b in m.items():
            if lo <= b <= hi:
                rs.append((a, a))
    return rs


_JPOSIX = {"ALPHA", "LOWER", "UPPER", "SPACE", "PUNCT", "XDIGIT", "ALNUM", "CNTRL", "DIGIT", "BLANK", "GRAPH",
           "PRINT"}


def _prop_ranges(name: str, ci: bool, uclass: bool):
    """Java Pattern.family: \\p{name} -> code-point ranges (raises UnsupportedJavaRegex if unknown)."""
    def get(key):
        rs = _uset(key)
        return list(rs) if rs else None

    def gc(nm):
        return (get("gci:" + nm) if ci else None) or get("gc:" + nm)

    def uprop(nm):
        nm = nm.upper()
        return (get("upi:" + nm) if ci else None) or get("up:" + nm)

    def script(nm):
        r = get("sc:" + nm.upper())
        if r is None:
            raise UnsupportedJavaRegex("Unknown character script name {%s}" % nm)
        return r

    def block(nm):
        r = get("blk:" + nm.upper())
        if r is None:
            raise UnsupportedJavaRegex("Unknown character block name {%s}" % nm)
        return r

    if "=" in name:
        k, v = name.split("=", 1)
        k = k.lower()
        if k in ("sc", "script"):
            return script(v)
        if k in ("blk", "block"):
            return block(v)
        if k in ("gc", "general_category") and gc(v) is not None:
            return gc(v)
        raise UnsupportedJavaRegex("Unknown Unicode property {%s}" % name)
    if name.startswith("In"):
        return block(name[2:])
    if name.startswith("Is"):
        r = uprop(name[2:]) or gc(name[2:])
        return r if r is not None else script(name[2:])
    if uclass and name.upper() in _JPOSIX:
        return uprop(name)
    r = gc(name)
    if r is None:
        raise UnsupportedJavaRegex("Unknown character property name {%s}" % name)
    return r


def _escape_ranges(e: str, uclass: bool):
    """(ranges, negated) of a predefined class escape letter."""
    low = e.lower()
    if low == "d":
        rs = list(_uset("u:digit")) if uclass else [(48, 57)]
    elif low == "s":
        rs = list(_uset("u:space")) if uclass else [(9, 13), (32, 32)]
    elif low == "w":
        rs = list(_uset("u:word")) if uclass else [(48, 57), (65, 90), (95, 95), (97, 122)]
    elif low == "h":
        rs = [(0x20, 0x20), (9, 9), (0xA0, 0xA0), (0x1680, 0x1680), (0x180E, 0x180E), (0x2000, 0x200A),
              (0x202F, 0x202F), (0x205F, 0x205F), (0x3000, 0x3000)]
    else:  # v
        rs = [(0x0A, 0x0D), (0x85, 0x85), (0x2028, 0x2029)]
    return rs, e.isupper()


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


def _prop_name(p: str, i: int):
    """p[i] is 'p' or 'P'. Returns (name, negated, new_i)."""
    neg = p[i] == "P"
    if i + 1 >= len(p):
        raise UnsupportedJavaRegex("Illegal character family")
    if p[i + 1] == "{":
        j = p.find("}", i + 2)
        if j < 0:
            raise UnsupportedJavaRegex("Unclosed character family")
        name = p[i + 2:j]
        ni = j + 1
    else:
        name = p[i + 1]
        ni = i + 2
    if name.startswith("^"):
        neg = not neg
        name = name[1:]
    return name, neg, ni


def _char_escape_cp(p: str, i: int):
    """Java single-char escape at p[i] (after the backslash) -> (code point, new_i) or None."""
    c = p[i]
    simple = {"t": 9, "n": 10, "r": 13, "f": 12, "a": 7, "e": 27}
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
        if int(digs, 8) > 0o377:
            digs = digs[:-1]
            j -= 1
        return int(digs, 8), j
    if c == "x":
        if i + 1 < len(p) and p[i + 1] == "{":
            j = p.index("}", i + 2)
            return int(p[i + 2:j], 16), j + 1
        return int(p[i + 1:i + 3], 16), i + 3
    if c == "u":
        v = int(p[i + 1:i + 5], 16)
        j = i + 5
        if 0xD800 <= v < 0xDC00 and p.startswith("\\u", j):
            lo = int(p[j + 2:j + 6], 16)
            if 0xDC00 <= lo < 0xE000:
                return 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00), j + 6
        return v, j
    if c == "c":
        return ord(p[i + 1]) ^ 64, i + 2
    if not c.isalnum():
        return ord(c), i + 1
    return None


def _lit(cp: int, sc) -> str:
    """One literal code point under the scope's case flags."""
    if sc["i"] and (sc["u"] or sc["U"]):
        v = _case_variants(cp, True)
        if len(v) > 1:
            return _emit([(x, x) for x in v])
    return _re.escape(chr(cp))


def _word_boundary(neg: bool) -> str:
    """Unicode \\b / \\B ((?U)): Java's WORD predicate on both sides."""
    w = _emit(list(_uset("u:word")))
    if neg:
        return "(?:(?<=%s)(?=%s)|(?<!%s)(?!%s))" % (w, w, w, w)
    return "(?:(?<=%s)(?!%s)|(?<!%s)(?=%s))" % (w, w, w, w)


@functools.lru_cache(maxsize=65536)
def to_python(pattern: str) -> str:
    p = pattern
    out = []
    # scope stack: dict(dotall, multiline, unix, comments, ci, unicode case, unicode class, pending closes)
    scopes = [dict(s=False, m=False, d=False, x=False, i=False, u=False, U=False, close=0)]
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
            elif ch in "idmsuxUc":
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
            if ch in "smdxiu":
                s[ch] = v
            elif ch == "U":
                s["U"] = s["u"] = v          # UNICODE_CHARACTER_CLASS implies UNICODE_CASE
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
                out.append("".join(_lit(ord(ch), sc) for ch in lit))
                i = n if j < 0 else j + 2
                continue
            if e in "dDsSwWhHvV":
                rs, neg = _escape_ranges(e, sc["U"])
                out.append(_emit(rs, neg))
                i += 1
                continue
            if e in "pP":
                name, neg, i = _prop_name(p, i)
                out.append(_emit(_prop_ranges(name, sc["i"], sc["U"]), neg))
                continue
            if e in "bB":
                out.append(_word_boundary(e == "B") if sc["U"] else "\\" + e)
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
            r = _char_escape_cp(p, i)
            if r is None:
                raise UnsupportedJavaRegex("unknown escape \\%s" % e)
            out.append(_lit(r[0], sc))
            i = r[1]
            continue
        if c == "[":
            rs, i = _class_set(p, i, sc)
            out.append(_emit(rs))
            continue
        if c == ".":
            out.append("(?s:.)") if sc["s"] else out.append(DOT_UNIX if sc["d"] else DOT)
            i += 1
            continue
        if c == "$":
            if sc["m"]:
                out.append(r"(?=\n|\Z)" if sc["d"] else EOL_MULTI)
            else:
                out.append(EOL_UNIX if sc["d"] else EOL)
            i += 1
            continue
        if c == "^":
            if sc["m"]:
                out.append(r"(?:\A|(?<=\n))(?!\Z)" if sc["d"] else BOL_MULTI)
            else:
                out.append("\\A")
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
        out.append(c if c in "*+?" else _lit(ord(c), sc))
        i += 1
    out.append(")" * cur()["close"])
    return "".join(out)


def _class_set(p: str, i: int, sc):
    """Java character class at p[i] == '[' -> (code-point ranges, new_i): nested unions, '&&'
    intersections, negation of the whole class, predefined / property escapes, ranges, and the
    scope's CASE_INSENSITIVE (ASCII or UNICODE_CASE) closure of literal characters and ranges."""
    assert p[i] == "["
    i += 1
    neg = False
    if i < len(p) and p[i] == "^":
        neg = True
        i += 1
    ci, uc, U = sc["i"], sc["u"] or sc["U"], sc["U"]
    cur_rs, acc = [], None
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
            sub, i = _class_set(p, i, sc)
            cur_rs += sub
            continue
        if c == "&" and p.startswith("&&", i):
            i += 2
            acc = _norm(cur_rs) if acc is None else _inter(acc, _norm(cur_rs))
            cur_rs = []
            continue
        if c == "\\":
            if i + 1 >= len(p):
                raise UnsupportedJavaRegex("bad class escape")
            e = p[i + 1]
            if e == "Q":
                j = p.find("\\E", i + 2)
                end = len(p) if j < 0 else j
                for ch in p[i + 2:end]:
                    cur_rs += [(v, v) for v in (_case_variants(ord(ch), uc) if ci else [ord(ch)])]
                i = len(p) if j < 0 else j + 2
                continue
            if e in "dDsSwWhHvV":
                rs, ng = _escape_ranges(e, U)
                cur_rs += _neg(_norm(rs)) if ng else rs
                i += 2
                continue
            if e in "pP":
                name, ng, i = _prop_name(p, i + 1)
                rs = _prop_ranges(name, ci, U)
                cur_rs += _neg(_norm(rs)) if ng else rs
                continue
            r = _char_escape_cp(p, i + 1)
            if r is None:
                raise UnsupportedJavaRegex("bad class escape")
            lo, i = r
        else:
            lo = ord(c)
            i += 1
        if i + 1 < len(p) and p[i] == "-" and p[i + 1] not in "][":
            i += 1
            if p[i] == "\\":
                r = _char_escape_cp(p, i + 1)
                if r is None:
                    raise UnsupportedJavaRegex("Illegal character range")
                hi, i = r
            else:
                hi = ord(p[i])
                i += 1
            if hi < lo:
                raise UnsupportedJavaRegex("Illegal character range")
            cur_rs += _ci_range(lo, hi, uc) if ci else [(lo, hi)]
        else:
            cur_rs += [(v, v) for v in (_case_variants(lo, uc) if ci else [lo])]
    res = _norm(cur_rs)
    if acc is not None:
        res = _inter(acc, res)
    if neg:
        res = _neg(res)
    return res, i


@functools.lru_cache(maxsize=65536)
def compile_java(pattern: str):
    """Compile a Java regex into a Python ``regex`` object with Java-equivalent semantics."""
    return _re.compile(to_python(pattern), _re.ASCII | _re.V0)


def java_find(pattern: str, line: str) -> bool:
    return compile_java(pattern).search(line) is not None
