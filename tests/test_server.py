"""REST API parity with the reference (Parse.java:23-62) + service extras."""
import json
import math
import os

import pytest
import torch
import yaml
from fastapi.testclient import TestClient

from log_parser_amd import golden
from log_parser_amd.serve.app import create_app
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log


@pytest.fixture(scope="module")
def lib_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("patterns")
    sets, trig = make_library(30, seed=5, n_sets=3)
    sub = d / "nested"
    sub.mkdir()
    for i, s in enumerate(sets):
        target = (sub if i == 2 else d) / f"set{i}.{'yaml' if i else 'yml'}"
        target.write_text(yaml.safe_dump(s.model_dump(by_alias=True, exclude_none=True)))
    (d / "broken.yaml").write_text("patterns: [unclosed")
    (d / "ignored.txt").write_text("not a pattern file")
    return str(d), trig


@pytest.fixture(scope="module")
def client(lib_dir):
    cfg = Config.load(overrides={"pattern.directory": lib_dir[0], "engine.device": "cpu",
                                 "engine.batch.max-wait-ms": 1.0})
    with TestClient(create_app(cfg)) as c:
        yield c


def test_invalid_requests(client):
    for body in [b"", b"null", b'{"logs": "x"}', b'{"pod": null, "logs": "x"}', b"{not json"]:
        r = client.post("/parse", content=body, headers={"content-type": "application/json"})
        assert r.status_code == 400
        assert r.json() == {"error": "Invalid PodFailureData provided"}


def test_non_json_content_type_is_415(client):
    body = b'{"pod":{},"logs":"x"}'
    for ct, code in [("text/plain", 415), ("application/x-www-form-urlencoded", 415),
                     ("application/json;charset=utf-8", 200), ("APPLICATION/JSON", 200)]:
        r = client.post("/parse", content=body, headers={"content-type": ct})
        assert r.status_code == code, ct
        if code == 415:
            assert r.json() == {"error": "Content-Type must be application/json"}


def test_parse_matches_golden(client, lib_dir):
    from log_parser_amd.models.library import load_pattern_directory
    sets = load_pattern_directory(lib_dir[0])
    assert len(sets) == 3   # broken.yaml skipped, .txt ignored, nested dir walked
    logs = make_log(1500, lib_dir[1], seed=8, hit_rate=0.06)
    client.delete("/admin/frequency")
    r = client.post("/parse", json={"pod": {"metadata": {"name": "p1"}}, "logs": logs})
    assert r.status_code == 200
    res = r.json()
    g = golden.analyze(logs, sets, ScoringParams(), golden.FrequencyTracker(ScoringParams()))
    assert res["summary"] == g["summary"]
    assert res["metadata"]["totalLines"] == g["metadata"]["totalLines"]
    assert res["metadata"]["patternsUsed"] == g["metadata"]["patternsUsed"]
    assert len(res["analysisId"]) == 36
    assert len(res["events"]) == len(g["events"]) > 0
    for a, b in zip(res["events"], g["events"]):
        assert a["lineNumber"] == b["lineNumber"]
        assert a["matchedPattern"] == b["matchedPattern"]
        assert a["context"] == b["context"]
        assert math.isclose(a["score"], b["score"], rel_tol=1e-12)


def test_health_ready_metrics_admin(client):
    assert client.get("/health").json()["status"] == "UP"
    rd = client.get("/ready").json()
    assert rd["status"] == "UP" and rd["library"]["patterns"] == 30
    client.post("/parse", json={"pod": {}, "logs": "nothing to see"})
    m = client.get("/metrics").text
    assert "lp_requests_total" in m and "lp_batches_total" in m
    stats = client.get("/admin/frequency").json()
    assert isinstance(stats, dict)
    assert client.delete("/admin/frequency").json() == {"reset": "all"}
    assert client.get("/admin/frequency/nope").status_code == 404


def test_concurrent_requests_are_batched(client, lib_dir):
    import concurrent.futures as cf
    logs = [make_log(200, lib_dir[1], seed=100 + i, hit_rate=0.05) for i in range(24)]
    with cf.ThreadPoolExecutor(8) as ex:
        rs = list(ex.map(lambda l: client.post("/parse", json={"pod": {"metadata": {"name": "x"}}, "logs": l}), logs))
    assert all(r.status_code == 200 for r in rs)
    m = client.get("/metrics").text
    batches = int([l for l in m.splitlines() if l.startswith("lp_batches_total")][0].split()[1])
    reqs = int([l for l in m.splitlines() if l.startswith("lp_batched_requests_total")][0].split()[1])
    assert reqs >= 24 and batches <= reqs


def test_missing_pattern_directory_tolerated(tmp_path):
    cfg = Config.load(overrides={"pattern.directory": str(tmp_path / "nope"), "engine.device": "cpu"})
    with TestClient(create_app(cfg)) as c:
        r = c.post("/parse", json={"pod": {}, "logs": "a\nb\n"})
        assert r.status_code == 200
        j = r.json()
        assert j["events"] == [] and j["summary"]["highestSeverity"] == "NONE" and j["metadata"]["totalLines"] == 2


def test_match_logging(caplog):
    import logging
    from log_parser_amd import LogParser
    sets, trig = make_library(5, seed=2)
    lp = LogParser(sets, config=Config.load(overrides={"engine.device": "cpu", "server.log-matches": "true"}))
    with caplog.at_level(logging.DEBUG, logger="log_parser_amd.engine"):
        r = lp.parse(make_log(200, trig, seed=3, hit_rate=0.2))
    msgs = [m for m in caplog.messages if "Found match for pattern" in m]
    assert len(msgs) == len(r["events"]) > 0
    assert any("Chronological Factor=" in m for m in caplog.messages)


def test_stage_timings_opt_in(tmp_path):
    """engine.trace=true adds metadata.stageTimingsMs; default responses are unchanged."""
    import json as _json
    import torch
    from log_parser_amd.engine import Engine
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.utils.config import Config, ScoringParams
    from log_parser_amd.utils.synth import make_library, make_log
    sets, trig = make_library(10, seed=5)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(200, trig, seed=6, hit_rate=0.1)
    on = Engine(lib, Config.load(overrides={"engine.device": "cpu", "engine.trace": "true"}), device=torch.device("cpu"))
    off = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    a = _json.loads(on.analyze_batch_json([logs, logs])[0])
    b = _json.loads(off.analyze_batch_json([logs])[0])
    st = a["metadata"]["stageTimingsMs"]
    for k in ("line_index", "h2d", "prefilter", "verify_csr", "events_context_freq", "score", "d2h"):
        assert k in st and st[k] >= 0.0, (k, st)
    assert st["batchRequests"] == 2
    assert "stageTimingsMs" not in b["metadata"]
    assert [e["lineNumber"] for e in a["events"]] == [e["lineNumber"] for e in b["events"]]


def test_parse_special_characters_roundtrip(client, lib_dir):
    """Context lines with quotes, backslashes, control characters and non-ASCII text survive the
    native JSON emitter (csrc/io/json_emit.cpp) exactly."""
    from log_parser_amd.models.library import load_pattern_directory
    sets = load_pattern_directory(lib_dir[0])
    base = make_log(400, lib_dir[1], seed=9, hit_rate=0.1).split("\n")
    junk = [' "quoted" ', "back\\slash", "\ttab", "\x01\x1f\x7f", "é日本😀", "\\\"", "\b\f"]
    logs = "\n".join(l + junk[i % len(junk)] for i, l in enumerate(base))
    client.delete("/admin/frequency")
    r = client.post("/parse", json={"pod": {"metadata": {"name": "p2"}}, "logs": logs})
    assert r.status_code == 200
    res = r.json()
    g = golden.analyze(logs, sets, ScoringParams(), golden.FrequencyTracker(ScoringParams()))
    assert len(res["events"]) == len(g["events"]) > 0
    for a, b in zip(res["events"], g["events"]):
        assert a["context"] == b["context"]


def test_embedding_api_submit_file_resident_and_frequency(tmp_path):
    """api.LogParser beyond a facade: concurrent submit through the batcher (results equal the
    sequential golden model in submission order), parse_file (doc and stream), a resident log
    re-analysed, the compile report, and the FrequencyTrackingService surface."""
    import concurrent.futures as cf
    from log_parser_amd import LogParser, golden
    from log_parser_amd.utils.synth import make_library, make_log
    p = ScoringParams(freq_threshold=1.0)
    sets, trig = make_library(20, seed=77)
    cfg = Config.load(overrides={"engine.device": "cpu", "scoring.frequency.threshold": "1.0"})
    lp = LogParser(sets, config=cfg)
    reqs = [make_log(150, trig, seed=700 + i, hit_rate=0.1) for i in range(12)]
    futs = [lp.submit(r) for r in reqs]                       # submission order = frequency order
    outs = [json.loads(f.result(timeout=120)) for f in futs]
    tr = golden.FrequencyTracker(p)
    for r, o in zip(reqs, outs):
        g = golden.analyze(r, sets, p, tr)
        assert [e["score"] for e in o["events"]] == pytest.approx([e["score"] for e in g["events"]], rel=1e-12)
    stats = lp.frequency_statistics()
    assert stats and lp.pattern_frequency(next(iter(stats)))["currentCount"] == stats[next(iter(stats))]
    lp.reset_pattern_frequency(next(iter(stats)))
    assert lp.pattern_frequency(next(iter(stats)))["currentCount"] == 0
    lp.reset_all_frequencies()
    assert lp.frequency_statistics() == {}
    f = tmp_path / "x.log"
    f.write_text(make_log(3000, trig, seed=701, hit_rate=0.05))
    doc = lp.parse_file(str(f), stream=False)
    lp.reset_all_frequencies()
    st = lp.parse_file(str(f), stream=True, topk=5)
    assert st.total_lines == doc["metadata"]["totalLines"] and st.summary == doc["summary"]
    res = lp.load_resident(f.read_bytes(), chunk_bytes=16384)
    lp.reset_all_frequencies()
    again = lp.analyze_resident(res, topk=5)
    assert again.summary == st.summary and list(again.topk_line) == list(st.topk_line)
    rep = lp.validate()
    assert rep["library"]["patterns"] == 20 and rep["problems"] == []
    lp.close()
