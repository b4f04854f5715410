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
