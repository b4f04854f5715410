"""Generate csrc/regex/unicode_tables.inc: the Unicode sets java.util.regex resolves by name.

Run offline at development time (the output is committed; the build never runs this):

    python tools/gen_unicode_tables.py

Sources: the ``regex`` module's Unicode database (properties, categories, scripts, blocks; Unicode
15.x, the version Java 21's Character tables implement) and, for the NAME lists only, perl's
unicore files (``To/Sc.pl`` script names, ``UCD.pl`` script aliases, ``Blocks.txt`` block names)
plus the scripts / blocks added in Unicode 14 and 15. Case pairs come from Python's ``str.upper``
/ ``str.lower`` (single-code-point results only = Java's simple case mappings).

Every set is keyed the way jregex.cpp resolves ``\\p{..}`` (mirroring java.util.regex.Pattern.family
and CharPredicates): ``gc:`` forProperty names (case-sensitive, ``gci:`` their CASE_INSENSITIVE
variants), ``up:`` forUnicodeProperty / forPOSIXName names (upper-cased, ``upi:`` case-insensitive
variants), ``sc:`` script names and aliases, ``blk:`` block names in Java's three accepted forms,
``u:`` the UNICODE_CHARACTER_CLASS predicates behind ``\\w \\d \\s`` and ``\\b``.
"""
from __future__ import annotations

import os
import re
import sys
import unicodedata

import regex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "csrc", "regex", "unicode_tables.inc")
UNICORE = "/usr/share/perl/5.34.0/unicore"
MAXCP = 0x10FFFF
ALL = "".join(chr(c) for c in range(MAXCP + 1))

NEW_SCRIPTS = {"Cypro_Minoan": "Cpmn", "Old_Uyghur": "Ougr", "Tangsa": "Tnsa", "Toto": "Toto",
               "Vithkuqi": "Vith", "Kawi": "Kawi", "Nag_Mundari": "Nagm"}
NEW_BLOCKS = ["Arabic Extended-B", "Vithkuqi", "Latin Extended-F", "Old Uyghur",
              "Unified Canadian Aboriginal Syllabics Extended-A", "Cypro-Minoan", "Tangsa", "Kana Extended-B",
              "Znamenny Musical Notation", "Latin Extended-G", "Toto", "Ethiopic Extended-B",
              "Arabic Extended-C", "Devanagari Extended-A", "Kawi", "Kaktovik Numerals", "Cyrillic Extended-D",
              "Nag Mundari", "CJK Unified Ideographs Extension H"]
# Character.UnicodeBlock names kept for compatibility with older Unicode versions
BLOCK_ALIASES = {"GREEK": "Greek and Coptic", "CYRILLIC_SUPPLEMENTARY": "Cyrillic Supplement",
                 "COMBINING_MARKS_FOR_SYMBOLS": "Combining Diacritical Marks for Symbols"}


def rx(prop: str):
    """Ranges [(lo, hi)] of a regex-module property expression."""
    return [(m.start(), m.end() - 1) for m in regex.finditer(prop + "+", ALL)]


def norm(rs):
    rs = sorted(rs)
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + 1:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def union(*sets):
    return norm([r for s in sets for r in s])


def minus(a, b):
    bits = bytearray(MAXCP + 2)
    for lo, hi in a:
        bits[lo:hi + 1] = b"\x01" * (hi - lo + 1)
    for lo, hi in b:
        bits[lo:hi + 1] = b"\x00" * (hi - lo + 1)
    return from_bits(bits)


def from_bits(bits):
    out, c = [], 0
    n = MAXCP + 1
    while c < n:
        if bits[c]:
            s = c
            while c < n and bits[c]:
                c += 1
            out.append((s, c - 1))
        else:
            c += 1
    return out


def pred(f):
    return from_bits(bytearray(1 if f(c) else 0 for c in range(MAXCP + 1)) + b"\x00")


def gc(*cats):
    return union(*[rx(r"\p{gc=%s}" % c) for c in cats])


def ascii_pred(f):
    return pred(lambda c: c < 128 and f(chr(c)))


def main():
    S = {}
    cats = ["Cn", "Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Me", "Mc", "Nd", "Nl", "No", "Zs", "Zl", "Zp", "Cc", "Cf",
            "Co", "Cs", "Pd", "Ps", "Pe", "Pc", "Po", "Sm", "Sc", "Sk", "So", "Pi", "Pf"]
    G = {c: gc(c) for c in cats}
    L = union(G["Lu"], G["Ll"], G["Lt"], G["Lm"], G["Lo"])
    LC = union(G["Lu"], G["Ll"], G["Lt"])
    for c in cats:
        S["gc:" + c] = G[c]
    S["gc:L"] = L
    S["gc:M"] = union(G["Mn"], G["Mc"], G["Me"])
    S["gc:N"] = union(G["Nd"], G["Nl"], G["No"])
    S["gc:Z"] = union(G["Zs"], G["Zl"], G["Zp"])
    S["gc:C"] = union(G["Cc"], G["Cf"], G["Co"], G["Cs"], G["Cn"])
    S["gc:P"] = union(*[G[c] for c in ("Pd", "Ps", "Pe", "Pc", "Po", "Pi", "Pf")])
    S["gc:S"] = union(G["Sm"], G["Sc"], G["Sk"], G["So"])
    S["gc:LC"] = LC
    S["gc:LD"] = union(L, G["Nd"])
    S["gc:L1"] = [(0, 0xFF)]
    S["gc:all"] = [(0, MAXCP)]
    for c in ("Lu", "Ll", "Lt"):
        S["gci:" + c] = LC
    # POSIX (ASCII) classes of forProperty
    punct = "!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~"
    S["gc:ASCII"] = [(0, 0x7F)]
    S["gc:Alnum"] = ascii_pred(str.isalnum)
    S["gc:Alpha"] = ascii_pred(str.isalpha)
    S["gc:Blank"] = [(9, 9), (32, 32)]
    S["gc:Cntrl"] = [(0, 0x1F), (0x7F, 0x7F)]
    S["gc:Digit"] = [(0x30, 0x39)]
    S["gc:Graph"] = ascii_pred(lambda ch: ch.isalnum() or ch in punct)
    S["gc:Lower"] = [(0x61, 0x7A)]
    S["gc:Print"] = [(0x20, 0x7E)]
    S["gc:Punct"] = ascii_pred(lambda ch: ch in punct)
    S["gc:Space"] = [(9, 13), (32, 32)]
    S["gc:Upper"] = [(0x41, 0x5A)]
    S["gc:XDigit"] = ascii_pred(lambda ch: ch in "0123456789abcdefABCDEF")
    S["gci:Lower"] = S["gci:Upper"] = S["gc:Alpha"]
    # Unicode binary properties (forUnicodeProperty) and the Unicode POSIX classes
    alpha = rx(r"\p{Alphabetic}")
    lower = rx(r"\p{Lowercase}")
    upper = rx(r"\p{Uppercase}")
    title = G["Lt"]
    white = rx(r"\p{White_Space}")
    digit = G["Nd"]
    hexd = union(digit, [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66), (0xFF10, 0xFF19), (0xFF21, 0xFF26), (0xFF41, 0xFF46)])
    join = [(0x200C, 0x200D)]
    word = union(alpha, G["Mn"], G["Me"], G["Mc"], digit, G["Pc"], join)
    cased = union(lower, upper, title)
    graph = minus([(0, MAXCP)], union(G["Zs"], G["Zl"], G["Zp"], G["Cc"], G["Cs"], G["Cn"]))
    blank = union(G["Zs"], [(9, 9)])
    up = {
        "ALPHABETIC": alpha, "ASSIGNED": minus([(0, MAXCP)], G["Cn"]), "CONTROL": G["Cc"],
        "EMOJI": rx(r"\p{Emoji}"), "EMOJI_PRESENTATION": rx(r"\p{Emoji_Presentation}"),
        "EMOJI_MODIFIER": rx(r"\p{Emoji_Modifier}"), "EMOJI_MODIFIER_BASE": rx(r"\p{Emoji_Modifier_Base}"),
        "EMOJI_COMPONENT": rx(r"\p{Emoji_Component}"), "EXTENDED_PICTOGRAPHIC": rx(r"\p{Extended_Pictographic}"),
        "HEXDIGIT": hexd, "HEX_DIGIT": hexd, "IDEOGRAPHIC": rx(r"\p{Ideographic}"),
        "JOINCONTROL": join, "JOIN_CONTROL": join, "LETTER": L, "LOWERCASE": lower,
        "NONCHARACTERCODEPOINT": pred(lambda c: (c & 0xFFFE) == 0xFFFE or 0xFDD0 <= c <= 0xFDEF),
        "TITLECASE": title, "PUNCTUATION": S["gc:P"], "UPPERCASE": upper, "WHITESPACE": white,
        "WHITE_SPACE": white, "WORD": word,
        # POSIX names (forPOSIXName with UNICODE_CHARACTER_CLASS, and the \p{IsAlpha} fallback)
        "ALPHA": alpha, "LOWER": lower, "UPPER": upper, "SPACE": white, "PUNCT": S["gc:P"], "XDIGIT": hexd,
        "ALNUM": union(alpha, digit), "CNTRL": G["Cc"], "DIGIT": digit, "BLANK": blank, "GRAPH": graph,
        "PRINT": minus(union(graph, blank), G["Cc"]),
    }
    for k, v in up.items():
        S["up:" + k] = v
    for k in ("LOWERCASE", "UPPERCASE", "TITLECASE", "LOWER", "UPPER"):
        S["upi:" + k] = cased
    # java.lang.Character predicates
    ignorable = union([(0, 8), (0x0E, 0x1B), (0x7F, 0x9F)], G["Cf"])
    zsep = union(G["Zs"], G["Zl"], G["Zp"])
    jstart = union(L, G["Nl"], G["Sc"], G["Pc"])
    uistart = union(L, G["Nl"], rx(r"\p{Other_ID_Start}"))
    java = {
        "javaLowerCase": lower, "javaUpperCase": upper, "javaAlphabetic": alpha,
        "javaIdeographic": up["IDEOGRAPHIC"], "javaTitleCase": title, "javaDigit": digit,
        "javaDefined": up["ASSIGNED"], "javaLetter": L, "javaLetterOrDigit": union(L, digit),
        "javaJavaIdentifierStart": jstart,
        "javaJavaIdentifierPart": union(jstart, digit, G["Mc"], G["Mn"], ignorable),
        "javaUnicodeIdentifierStart": uistart,
        "javaUnicodeIdentifierPart": union(uistart, G["Mn"], G["Mc"], digit, G["Pc"],
                                           rx(r"\p{Other_ID_Continue}"), ignorable),
        "javaIdentifierIgnorable": ignorable, "javaSpaceChar": zsep,
        "javaWhitespace": union(minus(zsep, [(0xA0, 0xA0), (0x2007, 0x2007), (0x202F, 0x202F)]),
                                [(9, 13), (0x1C, 0x1F)]),
        "javaISOControl": [(0, 0x1F), (0x7F, 0x9F)], "javaMirrored": rx(r"\p{Bidi_Mirrored}"),
    }
    for k, v in java.items():
        S["gc:" + k] = v
    for k in ("javaLowerCase", "javaUpperCase", "javaTitleCase"):
        S["gci:" + k] = cased
    # UNICODE_CHARACTER_CLASS predicates (\w \d \s \b)
    S["u:word"], S["u:digit"], S["u:space"] = word, digit, white
    # scripts: full names (Character.UnicodeScript enum form) + ISO 15924 aliases
    names = set()
    with open(os.path.join(UNICORE, "To", "Sc.pl")) as f:
        body = f.read().split("END\n")[0].split("<<'END';\n")[-1]
    for line in body.splitlines():
        parts = line.split("\t")
        if len(parts) >= 3 and parts[2]:
            names.add(parts[2])
    names |= {"Unknown", "Common", "Inherited"}
    aliases = {}
    with open(os.path.join(UNICORE, "UCD.pl")) as f:
        for m in re.finditer(r"'sc=([a-z_]+)' => '([a-z_]+)'", f.read()):
            aliases.setdefault(m.group(1), m.group(2))
    for full in sorted(names) + sorted(NEW_SCRIPTS):
        loose = full.lower().replace("_", "")
        al = NEW_SCRIPTS.get(full) or aliases.get(loose)
        try:
            rs = rx(r"\p{Script=%s}" % full)
        except Exception as e:  # noqa: BLE001
            print("skip script", full, e, file=sys.stderr)
            continue
        S["sc:" + full.upper()] = rs
        if al:
            S["sc:" + al.upper()] = rs
    S.setdefault("sc:QAAI", S["sc:INHERITED"])
    # blocks: canonical name, name without spaces, enum form (spaces / hyphens -> '_'), upper-cased
    blocks = []
    with open(os.path.join(UNICORE, "Blocks.txt")) as f:
        for line in f:
            m = re.match(r"([0-9A-F]+)\.\.([0-9A-F]+); (.+)$", line.strip())
            if m:
                blocks.append((int(m.group(1), 16), int(m.group(2), 16), m.group(3)))
    for nm in NEW_BLOCKS:
        try:
            rs = rx(r"\p{Block=%s}" % nm.replace(" ", "_").replace("-", "_"))
        except Exception as e:  # noqa: BLE001
            print("skip block", nm, e, file=sys.stderr)
            continue
        if rs:
            blocks.append((rs[0][0], rs[-1][1], nm))
    by_name = {}
    for lo, hi, nm in blocks:
        rs = [(lo, hi)]
        by_name[nm] = rs
        for key in (nm.upper(), nm.upper().replace(" ", ""), re.sub(r"[ -]", "_", nm.upper())):
            S["blk:" + key] = rs
    for k, nm in BLOCK_ALIASES.items():
        S["blk:" + k] = by_name[nm]
    # simple case mappings (Character.toUpperCase / toLowerCase of one code point)
    upper_pairs, lower_pairs = [], []
    for c in range(MAXCP + 1):
        if 0xD800 <= c <= 0xDFFF:
            continue
        ch = chr(c)
        u, lw = ch.upper(), ch.lower()
        if len(u) == 1 and u != ch:
            upper_pairs.append((c, ord(u)))
        if len(lw) == 1 and lw != ch:
            lower_pairs.append((c, ord(lw)))
    write(S, upper_pairs, lower_pairs)


def write(S, upper_pairs, lower_pairs):
    keys = sorted(S)
    ranges, index = [], []
    dedup = {}
    for k in keys:
        rs = tuple(S[k])
        off = dedup.get(rs)
        if off is None:
            off = dedup[rs] = len(ranges) // 2
            for lo, hi in rs:
                ranges += [lo, hi]
        index.append((k, off, len(rs)))
    lines = ["// GENERATED by tools/gen_unicode_tables.py -- do not edit.",
             f"// Unicode data: regex module {regex.__version__} (Unicode property sets), Python "
             f"{unicodedata.unidata_version} case mappings.",
             "// Sets are sorted disjoint [lo, hi] code-point ranges; kUniSets is sorted by key.",
             "namespace lp { namespace uni {",
             f"static const uint32_t kRanges[{len(ranges)}] = {{"]
    for i in range(0, len(ranges), 16):
        lines.append("  " + ",".join("0x%X" % x for x in ranges[i:i + 16]) + ",")
    lines.append("};")
    lines.append("struct SetRef { const char* key; uint32_t off, n; };")
    lines.append(f"static const SetRef kSets[{len(index)}] = {{")
    for k, off, n in index:
        lines.append(f'  {{"{k}", {off}u, {n}u}},')
    lines.append("};")
    for name, pairs in (("kUpper", upper_pairs), ("kLower", lower_pairs)):
        flat = [x for p in pairs for x in p]
        lines.append(f"static const uint32_t {name}[{len(flat)}] = {{  // (code point, mapping) pairs")
        for i in range(0, len(flat), 16):
            lines.append("  " + ",".join("0x%X" % x for x in flat[i:i + 16]) + ",")
        lines.append("};")
    lines.append("}  // namespace uni")
    lines.append("}  // namespace lp")
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"{OUT}: {len(index)} sets, {len(ranges) // 2} ranges, {len(upper_pairs)} + {len(lower_pairs)} case pairs")


if __name__ == "__main__":
    main()
