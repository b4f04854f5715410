"""GPU (MI355X) end-to-end paths beyond the kernels: chunked streaming on the device == the
single-pass device analysis == the CPU backend; checkpoint/resume of a device stream; a failing
device batch served by the CPU fallback with shared frequency state; the native HTTP front end
over a GPU engine == golden."""
import http.client
import json

import numpy as np
import pytest
import torch

from log_parser_amd import golden
from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.parallel.stream import StreamAnalyzer
from log_parser_amd.serve.app import Batcher, Service
from log_parser_amd.serve.native_http import NativeHttpFrontend
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.metrics import Metrics
from log_parser_amd.utils.synth import make_library, make_log

pytestmark = pytest.mark.gpu


def _eng(lib, dev, **over):
    return Engine(lib, Config.load(overrides={"engine.device": str(dev), **over}), device=dev)


@pytest.mark.parametrize("chunk", [8192, 1 << 20])
def test_device_stream_equals_single_pass_and_cpu(gpu_device, chunk):
    sets, trig = make_library(40, seed=41, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    data = (make_log(4000, trig, seed=42, hit_rate=0.08, crlf_rate=0.2) + "\n\n\r\n").encode()
    e1 = _eng(lib, gpu_device)
    t, n = e1.stage_text(data)
    ls, ll = K.split_lines(t, n)
    ref = e1.run(t, n, ls, ll, Segments.single(ls.numel(), t.device), e1.freq_carry())
    out = StreamAnalyzer(_eng(lib, gpu_device), chunk_bytes=chunk, topk=7).run(data)
    cpu = StreamAnalyzer(_eng(lib, torch.device("cpu")), chunk_bytes=chunk, topk=7).run(data)
    assert out.total_lines == ls.numel() == cpu.total_lines
    gl, pat, score = out.events
    np.testing.assert_array_equal(gl, ref.ev_line.cpu().numpy())
    np.testing.assert_array_equal(pat, ref.ev_pat.cpu().numpy())
    np.testing.assert_allclose(score, ref.score.cpu().numpy(), rtol=1e-15, atol=0)
    for a, b in zip(out.events, cpu.events):
        np.testing.assert_array_equal(a, b) if a.dtype.kind != "f" else np.testing.assert_allclose(a, b, rtol=1e-13)
    assert out.summary == cpu.summary


def test_device_stream_checkpoint_resume_is_exact(gpu_device, tmp_path):
    sets, trig = make_library(30, seed=81, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    data = make_log(3000, trig, seed=82, hit_rate=0.08).encode()
    ref = StreamAnalyzer(_eng(lib, gpu_device), chunk_bytes=8192, topk=10).run(data)
    ck = str(tmp_path / "stream.ckpt.npz")
    eng = _eng(lib, gpu_device)
    with pytest.raises(RuntimeError, match="injected"):
        StreamAnalyzer(eng, chunk_bytes=8192, topk=10).run(data, checkpoint=ck, fail_after_chunks=5)
    out = StreamAnalyzer(eng, chunk_bytes=8192, topk=10).run(data, checkpoint=ck, resume=ck)
    assert out.chunks == ref.chunks and out.total_lines == ref.total_lines
    for a, b in zip(out.events, ref.events):
        np.testing.assert_array_equal(a, b)
    assert out.summary == ref.summary


def test_gpu_batch_fault_falls_back_with_shared_frequency(gpu_device):
    sets, trig = make_library(20, seed=61)
    params = ScoringParams(freq_threshold=1.0)
    lib = CompiledLibrary(sets, params)
    eng = _eng(lib, gpu_device, **{"engine.fault-inject-every": "2"})
    m = Metrics()
    b = Batcher([eng], 1, 1 << 30, 0.0, m)
    reqs = [make_log(300, trig, seed=70 + i, hit_rate=0.06) for i in range(6)]
    outs = [json.loads(b.submit(r).result(timeout=300)) for r in reqs]     # one at a time: inline path
    b.close()
    assert m.device_failures == 3
    fz = golden.FrequencyTracker(params)
    for r, o in zip(reqs, outs):
        g = golden.analyze(r, sets, params, fz)
        assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
               [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]]
        assert o["summary"] == g["summary"]
        for a, c in zip(o["events"], g["events"]):
            assert a["score"] == pytest.approx(c["score"], rel=1e-12, abs=0)


def test_native_http_over_gpu_engine_equals_golden(gpu_device):
    sets, trig = make_library(15, seed=23)
    params = ScoringParams()
    lib = CompiledLibrary(sets, params)
    cfg = Config.load(overrides={"engine.device": str(gpu_device)})
    fe = NativeHttpFrontend(Service(cfg, Engine(lib, cfg, device=gpu_device)), "127.0.0.1", 0, io_threads=2)
    try:
        c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=120)
        fz = golden.FrequencyTracker(params)
        for i in range(5):
            logs = make_log(500 + 100 * i, trig, seed=300 + i, hit_rate=0.05, crlf_rate=0.1)
            c.request("POST", "/parse", body=json.dumps({"pod": {"metadata": {"name": f"p{i}"}}, "logs": logs}),
                      headers={"content-type": "application/json"})
            r = c.getresponse()
            assert r.status == 200
            o = json.loads(r.read())
            g = golden.analyze(logs, sets, params, fz)
            assert o["metadata"]["totalLines"] == g["metadata"]["totalLines"]
            assert [(e["lineNumber"], e["context"]) for e in o["events"]] == \
                   [(e["lineNumber"], e["context"]) for e in g["events"]]
            assert o["summary"] == g["summary"]
        # bodies of 300-500 KB: the logs text decoded by the IO thread while it arrives, into pinned
        # buffers the engine stages in place with the decoder's newline positions (DecodePool,
        # Engine._stage_docs); duplicates of the newline-heavy tail and CRLF lines included
        eng = fe.svc.engine()
        n0 = eng.inplace_stages
        for i in range(4):
            logs = make_log(3500 + 500 * i, trig, seed=400 + i, hit_rate=0.05, crlf_rate=0.1) + "\n\ntail é\u2028x"
            c.request("POST", "/parse", body=json.dumps({"pod": {"metadata": {"name": f"q{i}"}}, "logs": logs}),
                      headers={"content-type": "application/json"})
            r = c.getresponse()
            assert r.status == 200
            o = json.loads(r.read())
            g = golden.analyze(logs, sets, params, fz)
            assert o["metadata"]["totalLines"] == g["metadata"]["totalLines"]
            assert [(e["lineNumber"], e["context"]) for e in o["events"]] == \
                   [(e["lineNumber"], e["context"]) for e in g["events"]]
            assert [e["score"] for e in o["events"]] == pytest.approx([e["score"] for e in g["events"]], rel=1e-12)
            assert o["summary"] == g["summary"]
        assert eng.inplace_stages - n0 == 4
        c.close()
    finally:
        fe.close()
