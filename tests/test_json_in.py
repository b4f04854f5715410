"""Native /parse body decoder (csrc/io/json_in.cpp) against json.loads: same accept/reject decision,
same `pod` null check, same pod name and byte-identical `logs` for every body it does not hand
back to json.loads (status 3)."""
import json
import random

import pytest

from log_parser_amd.native import N


def _ref(body: bytes):
    try:
        d = json.loads(body)
    except ValueError:
        return (1,)
    if not isinstance(d, dict):
        return (2,)
    pod = d.get("pod")
    logs = d.get("logs")
    kind = 1 if isinstance(logs, str) else (0 if logs is None else 2)
    md = pod.get("metadata") if isinstance(pod, dict) else None
    name = md.get("name") if isinstance(md, dict) else None
    return (0, pod is not None, name if isinstance(name, str) else None, kind,
            logs.encode() if kind == 1 else None)


def _check(body: bytes, two_pass="one"):
    # "one": validate + decode in one pass into a string; "two": validate, then unescape the span;
    # "into": validate + decode into the caller's buffer (the HTTP IO thread's mode)
    got = N.parse_pod_request(body, two_pass == "two", two_pass == "into")
    if got[0] == 3:
        return False
    ref = _ref(body)
    if ref[0] != 0:
        assert got[0] == ref[0], (body[:200], got, ref)
    else:
        assert tuple(got) == ref, (body[:200], got, ref)
    return True


def _rand_str(rng):
    alphabet = ["a", "Z", " ", "\n", "\r\n", "\t", '"', "\\", "/", "é", "日本", " ", "\x01", "😀", "{", "]"]
    return "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 30)))


def _rand_value(rng, depth=0):
    k = rng.randrange(8 if depth < 4 else 5)
    if k == 0:
        return _rand_str(rng)
    if k == 1:
        return rng.choice([0, -1, 3.25, 1e-7, -2.5e10, 12345678901234567890])
    if k == 2:
        return rng.choice([True, False, None])
    if k == 3:
        return ""
    if k == 4:
        return rng.randint(-5, 5)
    if k == 5:
        return [_rand_value(rng, depth + 1) for _ in range(rng.randint(0, 4))]
    return {_rand_str(rng): _rand_value(rng, depth + 1) for _ in range(rng.randint(0, 4))}


@pytest.mark.parametrize("two_pass", ["one", "two", "into"])
@pytest.mark.parametrize("seed", range(4))
def test_native_decoder_matches_json_loads_on_random_requests(seed, two_pass):
    rng = random.Random(seed)
    native = 0
    for _ in range(600):
        d = {}
        for key in rng.sample(["pod", "logs", "events", "spec", "x"], rng.randint(0, 5)):
            if key == "pod":
                d[key] = rng.choice([None, {"metadata": {"name": _rand_str(rng)}}, {"metadata": None}, "s", [],
                                     {"metadata": {"name": 5, "labels": {"a": "b"}}}, {"spec": _rand_value(rng)}])
            elif key == "logs":
                d[key] = rng.choice([_rand_str(rng) * rng.randint(1, 50), None, 7, ["a"], ""])
            else:
                d[key] = _rand_value(rng)
        body = json.dumps(d, ensure_ascii=rng.random() < 0.5, indent=rng.choice([None, 1])).encode()
        if rng.random() < 0.2 and "logs" in d:       # duplicate key: the last one wins
            body = body[:-1] + b', "logs": "dup\\nlast"}'
        native += _check(body, two_pass)
        if rng.random() < 0.3:                        # corruptions must be rejected like json.loads
            cut = rng.randrange(len(body) + 1)
            native += _check(body[:cut], two_pass)
            native += _check(body + rng.choice([b"x", b",", b"}", b" ", b"\n"]), two_pass)
    assert native > 500                               # most bodies take the native path


def test_native_decoder_edge_cases():
    cases = [b"", b"   ", b"null", b"[]", b'"x"', b"{}", b'{"pod":{}}', b'{"pod":{},"logs":"a"}  \n',
             b'{"pod":{},"logs":"a\x01"}', b'{"pod":{},"logs":"\\q"}', b'{"pod":{},"logs":"\\u12"}',
             b'{"pod":{},"logs":"\\u00e9\\u20ac\\u0000"}', b'{"pod" {}}', b'{"pod":{},}', b'{"pod":01}',
             b'{"pod":1.}', b'{"pod":-}', b'{"pod":1e5,"logs":"x"}', b'{"pod":tru}', b'{"pod":{"metadata":{"name":""}},"logs":""}',
             b'{"logs":"a","pod":{"metadata":{"name":"n1"}},"pod":{"metadata":{}}}']
    for c in cases:
        assert _check(c), c
    for c in [b'{"pod":NaN}', b'{"pod":{},"logs":"\\ud83d\\ude00"}', b'\xef\xbb\xbf{}', b'{"pod":{},"logs":"\xff"}',
              b"[" * 600 + b"]" * 600]:
        assert N.parse_pod_request(c)[0] == 3, c      # handed to json.loads


@pytest.mark.parametrize("two_pass", ["one", "two", "into"])
def test_native_decoder_64_byte_blocks(two_pass):
    """Long logs go through the 64-byte branch-free block decoder (AVX-512 VBMI2 hosts): backslash
    runs of every length at every offset, runs crossing a block boundary, escaped quotes, a closing
    quote and invalid / \\u escapes inside a block -- all byte-identical to json.loads."""
    rng = random.Random(5)
    pieces = ["a" * 63, "x" * 64, "b", " ", "\\", "\\\\", "\\\\\\", "\\n", "\\t", "\\r", "\\/", '\\"',
              "\\b", "\\f", "\\u00e9", "\\u20ac", "\\q", "\x01", "\u00e9"]
    native = 0
    for _ in range(3000):
        raw = "z" * rng.randint(0, 130) + "".join(rng.choice(pieces) for _ in range(rng.randint(1, 24)))
        body = ('{"pod": {}, "logs": "' + raw + '"}').encode()
        native += _check(body, two_pass)
    assert native > 1000


def test_decoded_length_and_exact_decoder():
    """The front end counts each log's decoded length while validating (skip mode), and the
    packer's exact-bounds decoder (documents decoded side by side into one buffer) gives the same
    bytes as json.loads -- escapes and UTF-8 at every position around the decoder's prefix cut."""
    import json as _json
    import random
    from log_parser_amd.native import N
    rng = random.Random(7)
    atoms = ["a", "xyz ", "\n", "\r\n", '"', "\\", "/", "\t", "\b", "\f", "é", "€", "😀", "\u0085", " ",
             "\x01", "\x7f", "ß" * 3]
    for n in list(range(0, 40)) + list(range(370, 470)) + [1000, 5000, 20000]:
        s = "".join(rng.choice(atoms) for _ in range(n))
        for ensure_ascii in (False, True):
            body = _json.dumps({"pod": {}, "logs": s}, ensure_ascii=ensure_ascii).encode()
            st, off, ln, dlen = N.pod_logs_span(body)
            if ensure_ascii and "😀" in s:
                assert st == 3            # \ud83d\ude00: surrogate escapes go to json.loads
                continue
            assert st == 0
            want = s.encode("utf-8")
            assert dlen == len(want), (n, ensure_ascii)
            got, intact = N.decode_json_exact(body[off:off + ln])
            assert got == want and intact, (n, ensure_ascii)


def _stream_cuts(rng, n):
    """Arrival prefix lengths of an n-byte body: a few large reads, many tiny ones, or every byte."""
    k = rng.randrange(3)
    if k == 0:
        cuts = sorted(rng.sample(range(n + 1), min(n + 1, rng.randint(1, 12))))
    elif k == 1:
        cuts, c = [], 0
        while c < n:
            c += rng.randint(1, 300)
            cuts.append(min(c, n))
    else:
        cuts = list(range(0, n + 1, max(1, n // 400)))
    return cuts


@pytest.mark.parametrize("seed", range(6))
def test_logs_prefetch_while_arriving_equals_one_pass(seed):
    """The HTTP IO thread decodes a /parse body's logs string between reads (logs_prefetch) and the
    final parse resumes there: for any arrival pattern -- reads ending inside escapes, backslash runs,
    \\u escapes, UTF-8 sequences, before / inside / after the string -- the status, pod fields and
    decoded bytes equal the one-pass parse, and invalid bodies (also ones made invalid by the LAST
    byte) get the same verdict. Most valid bodies are really resumed (prefetch state >= 1)."""
    rng = random.Random(100 + seed)
    atoms = ["a" * 70, "line of text ", "\n", "\r\n", '"', "\\", "\\\\", "/", "\t", "é", "€", "😀", "日本",
             "\x7f", "z" * 130]
    resumed = 0
    for it in range(250):
        s = "".join(rng.choice(atoms) for _ in range(rng.randint(0, 160)))
        d = {}
        for key in rng.sample(["pod", "logs", "x"], 3):
            if key == "pod":
                d[key] = rng.choice([{"metadata": {"name": "p-" + str(it)}}, None, {"spec": _rand_value(rng)}])
            elif key == "logs":
                d[key] = s
            else:
                d[key] = _rand_value(rng)
        body = json.dumps(d, ensure_ascii=rng.random() < 0.3).encode()
        k = rng.random()
        if k < 0.1:                                   # invalid at the last byte
            body = body[:-1] + rng.choice([b"]", b",", b"x"])
        elif k < 0.15:                                # duplicate member after the string
            body = body[:-1] + b', "logs": "dup\\nlast"}'
        elif k < 0.2 and len(body) > 10:              # a control byte inside the string
            i = body.find(b'"logs"')
            if i >= 0:
                j = body.find(b'"', i + 7) + 1 + rng.randrange(max(1, len(s) // 2 + 1))
                body = body[:j] + b"\x01" + body[j:]
        want = N.parse_pod_request(body, False, True)
        got = N.parse_pod_request_stream(body, _stream_cuts(rng, len(body)))
        assert tuple(got[:5]) == tuple(want), (body[:120], got[:5], want)
        if want[0] == 0 and want[3] == 1 and got[5] >= 1:
            resumed += 1
    assert resumed > 50


def test_logs_prefetch_large_body_every_boundary():
    """A 200 KB log string (escapes every ~100 bytes, multi-byte characters, \\u escapes) arriving in
    reads of every length 1..67 bytes around its escapes decodes identically and is prefetched to its
    closing quote once the last read is in."""
    rng = random.Random(3)
    atoms = ["INFO service started ok ", "\n", "\r\n", "é", "€", "\\", '"', "\t", "😀", "\x00"]
    s = "".join(rng.choice(atoms) for _ in range(25_000))
    body = json.dumps({"pod": {"metadata": {"name": "big"}}, "logs": s}, ensure_ascii=False).encode()
    want = N.parse_pod_request(body, False, True)
    assert want[0] == 0 and want[4] == s.encode()
    for step in (1, 7, 64, 67, 4096, 65536):
        cuts = list(range(0, len(body), step)) if step > 1 else list(range(0, 3000)) + [len(body) - 1]
        got = N.parse_pod_request_stream(body, cuts)
        assert tuple(got[:5]) == tuple(want), step
        assert got[5] >= 1 and got[6] > len(body) // 2 if step > 1 else got[5] >= 1
    # \u escapes (ensure_ascii): reads ending inside the 4 hex digits
    body = json.dumps({"pod": {}, "logs": s.replace("😀", "")}, ensure_ascii=True).encode()
    want = N.parse_pod_request(body, False, True)
    for off in range(0, 12):
        got = N.parse_pod_request_stream(body, list(range(off, len(body), 61)))
        assert tuple(got[:5]) == tuple(want), off


def test_decoder_records_newline_positions():
    """The decoder records where it writes every '\\n' (escapes \\n and \\u000a, the block decoder's
    compressed output and the scalar path alike), so the packer skips its newline scan: the positions
    equal a scan of the decoded bytes for one-pass and prefetched (resumed) decodes."""
    rng = random.Random(11)
    atoms = ["x" * 61, "\n", "\n\n\n\n\n\n\n\n\n\n", "\r\n", "é", "😀", '"', "\\", "ab\ncd", "\t"]
    for it in range(300):
        s = "".join(rng.choice(atoms) for _ in range(rng.randint(0, 120)))
        body = json.dumps({"pod": {}, "logs": s}, ensure_ascii=rng.random() < 0.3).encode()
        if rng.random() < 0.3:
            body = body.replace(b"\\n", b"\\u000a", rng.randint(0, 5))
        got = N.parse_pod_request_stream(body, _stream_cuts(rng, len(body)) if it % 2 else [])
        if got[0] == 3:                               # surrogate-pair escapes: json.loads decides
            continue
        assert got[0] == 0 and got[4] == s.encode()
        assert list(got[7]) == [i for i, b in enumerate(got[4]) if b == 10], it
