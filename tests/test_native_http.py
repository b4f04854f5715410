"""Native HTTP/1.1 front end (csrc/io/http_server.cpp + serve/native_http.py): the reference's
REST contract (Parse.java:23-61) over real sockets -- 200 + AnalysisResult equal to the golden
model, 400 for null body/pod, keep-alive, pipelining, Expect: 100-continue, Connection: close,
413, chunked bodies, admin + metrics routes through the shared Service, concurrent clients."""
import http.client
import json
import socket
import threading

import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.serve.app import Service
from log_parser_amd.serve.native_http import NativeHttpFrontend
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


@pytest.fixture(scope="module")
def server():
    sets, trig = make_library(15, seed=23)
    lib = CompiledLibrary(sets, ScoringParams())
    cfg = Config.load(overrides={"engine.device": "cpu", "server.max-body-bytes": 4 << 20})
    eng = Engine(lib, cfg, device=torch.device("cpu"))
    fe = NativeHttpFrontend(Service(cfg, eng), "127.0.0.1", 0, io_threads=2)
    yield fe, sets, trig
    fe.close()


def _post(conn, body: bytes, headers=None):
    conn.request("POST", "/parse", body=body, headers={"content-type": "application/json", **(headers or {})})
    r = conn.getresponse()
    return r.status, r.read()


def test_parse_and_errors(server):
    fe, sets, trig = server
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=60)
    c.request("DELETE", "/admin/frequency")
    assert c.getresponse().read() == b'{"reset":"all"}'
    logs = make_log(800, trig, seed=24, hit_rate=0.05)
    tracker = golden.FrequencyTracker(ScoringParams())
    for _ in range(3):                                   # keep-alive: one connection, several requests
        st, out = _post(c, json.dumps({"pod": {"metadata": {"name": "p"}}, "logs": logs}).encode())
        assert st == 200
        o, g = json.loads(out), golden.analyze(logs, sets, ScoringParams(), tracker)
        assert o["summary"] == g["summary"] and len(o["events"]) == len(g["events"]) > 0
        assert [e["score"] for e in o["events"]] == pytest.approx([e["score"] for e in g["events"]], rel=1e-12)
    for body in [b"", b"null", b"[1]", b'{"logs":"x"}', b'{"pod":null,"logs":"x"}', b"{bad"]:
        assert _post(c, body) == (400, b'{"error":"Invalid PodFailureData provided"}'), body
    assert _post(c, b'{"pod":{},"logs":5}')[0] == 400
    st, out = _post(c, b'{"pod":{},"logs":"a\\ud83d\\ude00b","x":NaN}')    # json.loads fallback route
    assert st == 200 and json.loads(out)["metadata"]["totalLines"] == 1
    for path, code in [("/health", 200), ("/ready", 200), ("/admin/frequency", 200), ("/nope", 404)]:
        c.request("GET", path)
        r = c.getresponse()
        r.read()
        assert r.status == code, path
    c.request("GET", "/metrics")
    m = c.getresponse().read().decode()
    assert 'lp_requests_total{code="200"}' in m
    c.close()


def test_non_json_content_type_is_415(server):
    """@Consumes(MediaType.APPLICATION_JSON) (Parse.java:42): a non-JSON media type is refused
    before the body is looked at; parameters and case do not matter; no header is accepted."""
    fe, _, _ = server
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=60)
    body = b'{"pod":{},"logs":"x"}'
    for ct, code in [("text/plain", 415), ("application/xml", 415), ("application/jsonx", 415),
                     ("Application/JSON; charset=UTF-8", 200), ("application/json", 200)]:
        c.request("POST", "/parse", body=body, headers={"content-type": ct})
        r = c.getresponse()
        out = r.read()
        assert r.status == code, (ct, out)
        if code == 415:
            assert json.loads(out) == {"error": "Content-Type must be application/json"}
    c.request("POST", "/parse", body=body)          # http.client sends no Content-Type here
    r = c.getresponse()
    r.read()
    assert r.status == 200
    c.close()


def _raw(port, data: bytes, n_resp: int = 1, timeout=60):
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.sendall(data)
    buf = b""
    while buf.count(b"HTTP/1.1 ") < n_resp or not _complete(buf, n_resp):
        chunk = s.recv(1 << 16)
        if not chunk:
            break
        buf += chunk
    s.close()
    return buf


def _complete(buf: bytes, n: int) -> bool:
    pos, seen = 0, 0
    while seen < n:
        he = buf.find(b"\r\n\r\n", pos)
        if he < 0:
            return False
        head = buf[pos:he].decode(errors="replace").lower()
        if head.startswith("http/1.1 100"):
            pos = he + 4
            continue
        cl = [int(l.split(":")[1]) for l in head.split("\r\n") if l.startswith("content-length")]
        end = he + 4 + (cl[0] if cl else 0)
        if len(buf) < end:
            return False
        pos, seen = end, seen + 1
    return True


def test_pipelining_continue_close_limits(server):
    fe, _, trig = server
    body = json.dumps({"pod": {}, "logs": make_log(50, trig, seed=25)}).encode()
    req = (b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
           % len(body)) + body
    out = _raw(fe.port, req + b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n" + req, n_resp=3)
    assert out.count(b"HTTP/1.1 200 OK") == 3                      # pipelined, answered in order
    assert out.index(b'{"status":"UP"}') > out.index(b'"analysisId"')
    s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)      # Expect: 100-continue
    s.sendall((b"POST /parse HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\nContent-Length: %d\r\n\r\n" % len(body)))
    assert s.recv(1024).startswith(b"HTTP/1.1 100 Continue")
    s.sendall(body)
    got = b""
    while not _complete(got, 1):
        got += s.recv(1 << 16)
    assert got.startswith(b"HTTP/1.1 200 OK")
    s.close()
    out = _raw(fe.port, b"GET /health HTTP/1.1\r\nConnection: close\r\n\r\n")
    assert b"Connection: close" in out
    big = b"x" * 64
    out = _raw(fe.port, b"POST /parse HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % (5 << 20) + big)
    assert out.startswith(b"HTTP/1.1 413")
    out = _raw(fe.port, b"POST /parse HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 400")                          # decoded, then refused as JSON


def _chunked(body: bytes, sizes, ext: bool = False, trailers: bytes = b"") -> bytes:
    """`body` in Transfer-Encoding: chunked framing, chunk sizes cycling through `sizes`."""
    out, i, k = [], 0, 0
    while i < len(body):
        n = sizes[k % len(sizes)]
        k += 1
        part = body[i:i + n]
        i += n
        out.append(b"%x%s\r\n%s\r\n" % (len(part), b" ;name=\"v\"" if ext and k % 2 else b"", part))
    out.append(b"0\r\n" + trailers + b"\r\n")
    return b"".join(out)


def _strip(o):
    o.pop("analysisId")
    o["metadata"].pop("analyzedAt")
    o["metadata"].pop("processingTimeMs")
    return o


def _recv_responses(s, n):
    got = b""
    while not _complete(got, n):
        chunk = s.recv(1 << 16)
        if not chunk:
            break
        got += chunk
    out, pos = [], 0
    while len(out) < n:
        he = got.index(b"\r\n\r\n", pos)
        head = got[pos:he].decode()
        if head.startswith("HTTP/1.1 100"):
            pos = he + 4
            continue
        cl = int([l.split(":")[1] for l in head.lower().split("\r\n") if l.startswith("content-length")][0])
        out.append((int(head.split()[1]), got[he + 4:he + 4 + cl]))
        pos = he + 4 + cl
    return out


def test_chunked_bodies_equal_content_length(server):
    """Transfer-Encoding: chunked (Vert.x under Quarkus REST reads it: Parse.java:41-44, pom.xml:43-54):
    the same request framed by 1-byte, 4 KiB and mixed chunks -- with chunk extensions, trailer
    fields, a body delivered in slow segments, pipelined behind a chunked request -- answers the
    same AnalysisResult as the Content-Length request (ids and times stripped)."""
    import time
    fe, _, trig = server
    body = json.dumps({"pod": {"metadata": {"name": "ch"}}, "logs": make_log(120, trig, seed=26, hit_rate=0.1)}).encode()
    hdr = b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
    plain = hdr + b"Content-Length: %d\r\n\r\n" % len(body) + body

    def ask(raw, slow=False):
        _raw(fe.port, b"DELETE /admin/frequency HTTP/1.1\r\nHost: x\r\n\r\n")
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
        if slow:                                      # segments split mid size-line / mid CRLF
            for i in range(0, len(raw), 997):
                s.sendall(raw[i:i + 997])
                time.sleep(0.001)
        else:
            s.sendall(raw)
        (st, out), = _recv_responses(s, 1)
        s.close()
        return st, out

    st, ref = ask(plain)
    assert st == 200
    ref = _strip(json.loads(ref))
    assert ref["summary"]["significantEvents"] > 0
    cases = [
        hdr + b"Transfer-Encoding: chunked\r\n\r\n" + _chunked(body, [1]),
        hdr + b"Transfer-Encoding: chunked\r\n\r\n" + _chunked(body, [4096]),
        hdr + b"Transfer-Encoding: Chunked\r\n\r\n" + _chunked(body, [1, 7, 4096, 300, 2], ext=True,
                                                                 trailers=b"X-Sum: 1\r\nX-B: 2\r\n"),
        hdr + b"Transfer-Encoding: identity, chunked\r\nContent-Length: 5\r\n\r\n" + _chunked(body, [65536]),
        hdr + b"Transfer-Encoding: identity\r\nContent-Length: %d\r\n\r\n" % len(body) + body,
    ]
    for k, raw in enumerate(cases):
        st, out = ask(raw)
        assert st == 200, (k, out[:200])
        assert _strip(json.loads(out)) == ref, k
    st, out = ask(cases[2], slow=True)
    assert st == 200 and _strip(json.loads(out)) == ref
    # pipelined: chunked request, a GET, then a Content-Length request on one connection
    s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
    s.sendall(cases[0] + b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n" + plain)
    r = _recv_responses(s, 3)
    s.close()
    assert [x[0] for x in r] == [200, 200, 200] and r[1][1] == b'{"status":"UP"}'
    # Expect: 100-continue before a chunked body
    s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
    s.sendall(hdr + b"Transfer-Encoding: chunked\r\nExpect: 100-continue\r\n\r\n")
    assert s.recv(1024).startswith(b"HTTP/1.1 100 Continue")
    s.sendall(_chunked(body, [333]))
    (st, out), = _recv_responses(s, 1)
    s.close()
    assert st == 200 and "analysisId" in json.loads(out)


def test_large_body_decoded_while_arriving(server):
    """A >= 64 KiB /parse body is validated and decoded by the IO thread between reads (LogsPrefetch,
    server.prefetch-logs): delivered in slow segments that end inside escapes and multi-byte
    characters, it answers the same AnalysisResult as the body sent at once, and the prefetch really
    ran (stage counter). A body that becomes invalid only at its LAST byte still answers the
    reference's 400 (Parse.java:45-49) and records nothing in the frequency window."""
    import time
    fe, _, trig = server
    logs = make_log(2500, trig, seed=31, hit_rate=0.05) + '\n"quoted" \\ tab\t é€😀 end'
    body = json.dumps({"pod": {"metadata": {"name": "big"}}, "logs": logs}, ensure_ascii=False).encode()
    assert len(body) >= 64 << 10
    hdr = b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"

    def ask(b, seg=None):
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
        raw = hdr % len(b) + b
        if seg:
            i = 0
            while i < len(raw):
                n = seg[i % len(seg)]
                s.sendall(raw[i:i + n])
                i += n
                time.sleep(0.0005)
        else:
            s.sendall(raw)
        (st, out), = _recv_responses(s, 1)
        s.close()
        return st, out

    _raw(fe.port, b"DELETE /admin/frequency HTTP/1.1\r\nHost: x\r\n\r\n")
    st, ref = ask(body)
    assert st == 200
    ref = _strip(json.loads(ref))
    assert ref["summary"]["significantEvents"] > 0 and ref["metadata"]["totalLines"] == logs.count("\n") + 1
    before = fe.srv.stage_stats()["prefetched"]
    for seg in ([4093], [1, 2, 3, 997, 65536], [12289, 7, 8191]):
        _raw(fe.port, b"DELETE /admin/frequency HTTP/1.1\r\nHost: x\r\n\r\n")
        st, out = ask(body, seg)
        assert st == 200 and _strip(json.loads(out)) == ref, seg
    assert fe.srv.stage_stats()["prefetched"] >= before + 3
    # invalid at the last byte: 400, and the frequency window is exactly as before
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=60)
    c.request("GET", "/admin/frequency")
    win0 = c.getresponse().read()
    for bad in (body[:-1] + b"]", body[:-1], body + b"x"):
        st, out = ask(bad, [8191, 3])
        assert (st, out) == (400, b'{"error":"Invalid PodFailureData provided"}'), bad[-8:]
    c.request("GET", "/admin/frequency")
    assert c.getresponse().read() == win0
    c.close()


def test_chunked_errors(server):
    """Malformed chunked framing -> 400 (connection closed); a decoded size above
    server.max-body-bytes -> 413 (the encoded size does not count); codings other than chunked /
    identity -> 501; an invalid JSON body that arrived chunked -> the reference's 400."""
    fe, _, _ = server
    hdr = b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n"
    for bad in [b"zz\r\nhello\r\n0\r\n\r\n", b"5\r\nhelloXX0\r\n\r\n", b"5\nhello\r\n0\r\n\r\n",
                b"5 x\r\nhello\r\n0\r\n\r\n", b"1000000000000000\r\n", b"\r\n"]:
        out = _raw(fe.port, hdr + bad)
        assert out.startswith(b"HTTP/1.1 400"), (bad, out[:80])
        assert b"malformed chunked body" in out and b"Connection: close" in out
    big = (b"x" * 65536)
    # 64 x 64 KiB = 4 MiB decoded is allowed (4.2 MB encoded); one byte more is not
    out = _raw(fe.port, hdr + b"".join(b"10000\r\n" + big + b"\r\n" for _ in range(64)) + b"1\r\n")
    assert out.startswith(b"HTTP/1.1 413")
    out = _raw(fe.port, hdr + b"500000\r\n")                          # declared size alone is refused
    assert out.startswith(b"HTTP/1.1 413")
    for te in [b"gzip, chunked", b"deflate"]:
        out = _raw(fe.port, b"POST /parse HTTP/1.1\r\nTransfer-Encoding: " + te + b"\r\nContent-Length: 2\r\n\r\n{}")
        assert out.startswith(b"HTTP/1.1 501"), te
    out = _raw(fe.port, b"POST /parse HTTP/1.1\r\nTransfer-Encoding: chunked, chunked\r\n\r\n0\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 400")
    out = _raw(fe.port, hdr + _chunked(b'{"pod":null,"logs":"x"}', [3]))
    assert out.endswith(b'{"error":"Invalid PodFailureData provided"}')


def test_concurrent_clients(server):
    fe, _, trig = server
    logs = [make_log(100 + 10 * i, trig, seed=300 + i, hit_rate=0.05) for i in range(8)]
    nlines = [len(golden.split_lines(x)) for x in logs]
    errs = []

    def client(i):
        try:
            c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=120)
            for k in range(6):
                st, out = _post(c, json.dumps({"pod": {"metadata": {"name": f"c{i}"}}, "logs": logs[(i + k) % 8]}).encode())
                assert st == 200 and json.loads(out)["metadata"]["totalLines"] == nlines[(i + k) % 8]
            c.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=client, args=(i,)) for i in range(24)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs[:3]
    b = fe.svc.batcher()
    assert b.pipe.idle() and fe.svc.engine()._stage_pool._out == 0   # pipelined batches all released


def test_idle_connections_are_closed():
    sets, _ = make_library(5, seed=29)
    lib = CompiledLibrary(sets, ScoringParams())
    cfg = Config.load(overrides={"engine.device": "cpu", "server.idle-timeout-s": 0.5})
    fe = NativeHttpFrontend(Service(cfg, Engine(lib, cfg, device=torch.device("cpu"))), "127.0.0.1", 0, 1)
    try:
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=10)
        s.sendall(b"GET /health HTTP/1.1\r\n\r\n")
        assert b"200 OK" in s.recv(4096)
        s.settimeout(10)
        assert s.recv(4096) == b""                        # closed by the idle sweep (~0.5-1.5 s)
        s.close()
    finally:
        fe.close()


def test_raw_logs_unescaped_in_the_stage(server):
    """Direct mode drains /parse logs still JSON-escaped (N.RawLogs) and the packer unescapes them
    straight into the pinned stage: escapes of every kind, CRLF / CR-only lines, non-ASCII, a
    batch mixing raw and json.loads-fallback bodies, and RawLogs == their decode() through the
    engine."""
    from log_parser_amd.native import N
    fe, sets, trig = server
    base = make_log(300, trig, seed=31, hit_rate=0.05)
    logs = base.replace("\n", "\r\n", 40) + '\ttab "quoted" back\\slash caf\u00e9 \x01 end\n\n\n'
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=60)
    c.request("DELETE", "/admin/frequency")
    c.getresponse().read()
    st, out = _post(c, json.dumps({"pod": {"metadata": {"name": "raw"}}, "logs": logs}).encode())
    assert st == 200
    tracker = golden.FrequencyTracker(ScoringParams())
    o, g = json.loads(out), golden.analyze(logs, sets, ScoringParams(), tracker)
    assert o["metadata"]["totalLines"] == g["metadata"]["totalLines"]
    assert o["summary"] == g["summary"] and len(o["events"]) == len(g["events"]) > 0
    assert [e["context"] for e in o["events"]] == [e["context"] for e in g["events"]]

    # engine level: a RawLogs batch == the same logs as bytes (fresh frequency state each time)
    hs = N.HttpServer("127.0.0.1", 0, 1, 1 << 24, 60.0)
    try:
        bodies = [json.dumps({"pod": {}, "logs": l}).encode() for l in (logs, base, "")]
        socks = []
        for b in bodies:                  # connections stay open until the requests are drained
            s = socket.create_connection(("127.0.0.1", hs.port))
            s.sendall(b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                      b"Content-Length: %d\r\n\r\n" % len(b) + b)
            socks.append(s)
        got = []
        for _ in range(50):
            got += [r for r in hs.next_requests(8, 200, True) if r[1] == 0]
            if len(got) == 3:
                break
        for s in socks:
            s.close()
        assert len(got) == 3
        raws = sorted((r[2] for r in got), key=len, reverse=True)
        assert [r.decode() for r in raws] == [l.encode() for l in (logs, base, "")]
        eng = fe.svc.engine()
        eng.freq.reset_all()
        a = [json.loads(x) for x in eng.analyze_batch_json(raws)]
        eng.freq.reset_all()
        b = [json.loads(x) for x in eng.analyze_batch_json([logs.encode(), base.encode(), b""])]
        for x, y in zip(a, b):
            for r in (x, y):
                r.pop("analysisId"), r["metadata"].pop("analyzedAt"), r["metadata"].pop("processingTimeMs")
            assert x == y
        # mixed batch: raw + plain bytes
        eng.freq.reset_all()
        m = [json.loads(x) for x in eng.analyze_batch_json([raws[0], base.encode()])]
        assert m[0]["summary"] == a[0]["summary"] and m[1]["metadata"]["totalLines"] == a[1]["metadata"]["totalLines"]
    finally:
        hs.stop()


def test_load_generator_burst_over_many_connections(server):
    """The native load generator (config 5 over HTTP): 256 keep-alive connections established
    first, one request each fired together; every response is a complete 200 AnalysisResult."""
    import numpy as np
    from log_parser_amd.native import N
    fe, sets, trig = server
    msgs = []
    for k, n in enumerate((5, 40, 300)):
        body = json.dumps({"pod": {"metadata": {"name": f"p{k}"}}, "logs": make_log(n, trig, seed=90 + k)}).encode()
        msgs.append(b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: "
                    + str(len(body)).encode() + b"\r\n\r\n" + body)
    idx = np.arange(256, dtype=np.int32) % 3
    lat, st, wall, done = N.http_burst("127.0.0.1", fe.port, msgs, idx, 120.0)
    assert done == 256 and (st == 200).all() and (lat > 0).all() and wall >= lat.max() * 0.5


def _io_thread_cpus():
    """CPU lists of this process's native HTTP IO threads (named lp-io<k>)."""
    import os
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            if not name.startswith("lp-io"):
                continue
            with open(f"/proc/self/task/{tid}/status") as f:
                for line in f:
                    if line.startswith("Cpus_allowed_list:"):
                        out[name] = line.split(":", 1)[1].strip()
        except OSError:
            pass
    return out


def test_io_threads_widen_under_a_burst_and_narrow_back():
    """server.l3-affinity keeps the IO threads on one L3 (a lone /parse body is decoded by a helper
    core beside its IO thread), but a burst of connections needs every core: an IO thread holding more
    than `hi` connections moves to the wide CPU set, and back below `lo` (HttpServer.set_affinity_sets)."""
    import os
    import time
    from log_parser_amd.native import N
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 2:
        pytest.skip("needs two CPUs")
    narrow = allowed[:1]
    srv = N.HttpServer("127.0.0.1", 0, 1, 1 << 20)
    try:
        srv.set_affinity_sets(narrow, allowed, 4, 2)
        s0 = socket.create_connection(("127.0.0.1", srv.port), timeout=10)
        deadline = time.time() + 10
        while time.time() < deadline and _io_thread_cpus().get("lp-io0") != str(narrow[0]):
            time.sleep(0.05)
        assert _io_thread_cpus().get("lp-io0") == str(narrow[0])
        burst = [socket.create_connection(("127.0.0.1", srv.port), timeout=10) for _ in range(12)]
        deadline = time.time() + 10
        while time.time() < deadline and _io_thread_cpus().get("lp-io0") == str(narrow[0]):
            for s in burst:                           # traffic wakes the IO thread's loop
                s.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n")
            time.sleep(0.05)
        assert _io_thread_cpus().get("lp-io0") != str(narrow[0])
        for s in burst:
            s.close()
        deadline = time.time() + 10
        while time.time() < deadline and _io_thread_cpus().get("lp-io0") != str(narrow[0]):
            s0.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n")
            time.sleep(0.05)
        assert _io_thread_cpus().get("lp-io0") == str(narrow[0])
        s0.close()
    finally:
        srv.stop()


def test_arrival_slots_pipelined_expect_disconnect_and_exhaustion(server):
    """Large bodies go through the arrival slots (decoded on the helper core while they arrive):
    two pipelined in one write (the second one's bytes move the receive buffer while the first is
    registered), Expect: 100-continue, a client that disconnects mid-body (its slot and buffer are
    released: later bodies still prefetch), and more bodies in flight at once than there are slots
    (the rest decode on their IO thread) -- every response equal to the one-shot request's."""
    import time
    fe, _, trig = server
    hdr = b"POST /parse HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
    bodies = [json.dumps({"pod": {"metadata": {"name": f"a{i}"}},
                          "logs": make_log(900 + 37 * i, trig, seed=60 + i, hit_rate=0.05)}).encode() for i in range(3)]
    assert all(len(b) >= 64 << 10 for b in bodies)

    def reset():
        _raw(fe.port, b"DELETE /admin/frequency HTTP/1.1\r\nHost: x\r\n\r\n")

    refs = []
    for b in bodies:
        reset()
        (st, out), = _recv_responses(_conn_send(fe.port, hdr % len(b) + b), 1)
        assert st == 200
        refs.append(_strip(json.loads(out)))
    # two large requests pipelined in one write
    reset()
    s = _conn_send(fe.port, hdr % len(bodies[0]) + bodies[0] + hdr % len(bodies[1]) + bodies[1])
    r = _recv_responses(s, 2)
    s.close()
    assert [x[0] for x in r] == [200, 200]
    assert _strip(json.loads(r[0][1])) == refs[0]
    # (the second one saw the first one's record in the window: compare everything but the scores)
    o1 = _strip(json.loads(r[1][1]))
    assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o1["events"]] == \
           [(e["lineNumber"], e["matchedPattern"]["id"]) for e in refs[1]["events"]]
    # Expect: 100-continue, then the body in two halves
    reset()
    b = bodies[2]
    s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
    s.sendall((hdr % len(b)).replace(b"\r\n\r\n", b"\r\nExpect: 100-continue\r\n\r\n"))
    assert s.recv(1024).startswith(b"HTTP/1.1 100 Continue")
    s.sendall(b[:len(b) // 2])
    time.sleep(0.01)
    s.sendall(b[len(b) // 2:])
    (st, out), = _recv_responses(s, 1)
    s.close()
    assert st == 200 and _strip(json.loads(out)) == refs[2]
    # a client that leaves mid-body
    for _ in range(3):
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
        s.sendall(hdr % len(b) + b[:len(b) // 2])
        time.sleep(0.01)
        s.close()
    before = fe.srv.stage_stats()["prefetched"]
    reset()
    (st, out), = _recv_responses(_conn_send(fe.port, hdr % len(b) + b, slow=True), 1)
    assert st == 200 and _strip(json.loads(out)) == refs[2]
    assert fe.srv.stage_stats()["prefetched"] > before
    # more bodies in flight than arrival slots (32): all half-sent first, then completed
    socks = []
    for i in range(40):
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=60)
        s.sendall(hdr % len(bodies[0]) + bodies[0][:len(bodies[0]) // 2])
        socks.append(s)
    time.sleep(0.05)
    for s in socks:
        s.sendall(bodies[0][len(bodies[0]) // 2:])
    for s in socks:
        (st, out), = _recv_responses(s, 1)
        s.close()
        o = _strip(json.loads(out))
        assert st == 200
        assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
               [(e["lineNumber"], e["matchedPattern"]["id"]) for e in refs[0]["events"]]


def _conn_send(port, raw: bytes, slow: bool = False):
    import time
    s = socket.create_connection(("127.0.0.1", port), timeout=60)
    if slow:
        for i in range(0, len(raw), 8191):
            s.sendall(raw[i:i + 8191])
            time.sleep(0.0005)
    else:
        s.sendall(raw)
    return s


def test_burst_mode_bodies_reach_the_packer_undecoded():
    """server.io-decode-max-conns: above that many connections an IO thread stops decoding /parse
    bodies itself (under a burst it is the front's bottleneck) and the packer unescapes them. With
    the limit at 0 (and the arrival-time decode off) every body takes that route: large bodies --
    escapes, multi-byte characters, several on one keep-alive connection -- answer the same
    AnalysisResult as through the IO-thread decode with its arrival-time prefetch."""
    sets, trig = make_library(15, seed=23)
    logs = [make_log(n, trig, seed=40 + n, hit_rate=0.05) + '\n"q" \\ tab\t é€😀 end' for n in (60, 900, 2600)]
    bodies = [json.dumps({"pod": {"metadata": {"name": f"b{i}"}}, "logs": l}, ensure_ascii=False).encode()
              for i, l in enumerate(logs)]
    assert len(bodies[-1]) >= 64 << 10
    outs = {}
    for limit in (-1, 0):
        lib = CompiledLibrary(sets, ScoringParams())
        cfg = Config.load(overrides={"engine.device": "cpu", "server.max-body-bytes": 4 << 20,
                                     "server.io-decode-max-conns": limit, "server.prefetch-logs": limit != 0})
        eng = Engine(lib, cfg, device=torch.device("cpu"))
        fe = NativeHttpFrontend(Service(cfg, eng), "127.0.0.1", 0, io_threads=1)
        try:
            c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=60)
            res = []
            for b in bodies:
                st, out = _post(c, b)
                assert st == 200
                res.append(_strip(json.loads(out)))
            c.close()
            outs[limit] = res
            assert (fe.srv.stage_stats()["prefetched"] > 0) == (limit != 0)
        finally:
            fe.close()
    assert outs[0] == outs[-1]
    assert all(r["summary"]["significantEvents"] > 0 for r in outs[0])
