"""Command line (log_parser_amd/__main__.py): validate / analyze (whole-file and streamed)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = os.path.join(ROOT, "patterns", "examples", "k8s")


def _run(*args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "log_parser_amd", *args], capture_output=True, text=True,
                          env=env, cwd=ROOT, timeout=300)


def test_validate_reports_library(tmp_path):
    r = _run("validate", PAT)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["library"]["patterns"] > 0 and out["library"]["invalid"] == 0


def test_validate_flags_invalid(tmp_path):
    (tmp_path / "bad.yaml").write_text(
        "metadata: {library_id: bad, version: '1'}\n"
        "patterns:\n- id: p1\n  name: broken\n  severity: HIGH\n"
        "  primary_pattern: {regex: 'a(b', confidence: 0.5}\n")
    r = _run("validate", str(tmp_path))
    assert r.returncode == 1
    probs = json.loads(r.stdout)["problems"]
    assert any(p["kind"] == "invalid" and p["regex"] == "a(b" for p in probs)


@pytest.mark.parametrize("stream", [False, True])
def test_analyze_file(tmp_path, stream):
    log = tmp_path / "pod.log"
    log.write_text("starting\nERROR OOMKilled container app\nat com.x.Y.run(Y.java:1)\nback-off restarting failed container\n")
    args = ["analyze", str(log), "--patterns", PAT, "--device", "cpu"] + (["--stream"] if stream else [])
    r = _run(*args)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    if stream:
        assert out["totalLines"] == 4 and "summary" in out
    else:
        assert out["metadata"]["totalLines"] == 4 and "summary" in out
