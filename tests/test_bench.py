"""bench.py contract (the driver's scaling run): launched by torch.distributed.run with one rank
per device, rank 0 prints ONE JSON line whose value is the whole-job aggregate. Rehearsed here
with 2 CPU ranks over gloo (the 8-GPU RCCL run is the driver's)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_bench_json_contract(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--lines-per-gpu", "20000"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only, one line
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True and d["data"] == "synthetic"
    assert d["config"]["parallelism"] == "dp2"
    # whole-job aggregate: lines of BOTH ranks per second of the slowest rank
    assert d["config"]["global_batch"] == 2 * d["config"]["lines_per_gpu"]
    assert abs(d["value"] - d["config"]["global_batch"] / (d["ms_per_step"] / 1e3)) / d["value"] < 1e-3
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"].split(";")[0].strip()


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]            # rank 0 only, one line
    return json.loads(lines[0])


def test_bench_spawns_its_own_ranks(tmp_path):
    """``bench.py --gpus 3`` WITHOUT a launcher: the parent starts 3 rank processes itself (the
    driver's ``--gpus N`` contract), the JSON reports n_gpus 3 and the live world size."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--device", "cpu", "--steps", "2",
           "--warmup", "1", "--lines-per-gpu", "6000", "--block-lines", "6000", "--parse-requests", "0",
           "--library", "synthetic"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 3 and d["world_size"] == 3 and d["backend"] == "gloo"
    assert d["config"]["parallelism"] == "dp3" and len(d["ms_per_step_per_rank"]) == 3
    assert d["config"]["global_batch"] == 3 * d["config"]["lines_per_gpu"]
    assert d["ms_per_step"] == max(d["ms_per_step_per_rank"])
    assert d["config"]["events_to_host_rank0"] > 0


def test_bench_eight_ranks_cpu(tmp_path):
    """The driver's N=8 launch, rehearsed on CPU: 8 rank processes, gloo, halos on both sides of
    the 6 inner ranks, the two in-place collectives, per-rank diagnostics in the JSON."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--device", "cpu", "--steps", "2",
           "--warmup", "1", "--lines-per-gpu", "3000", "--block-lines", "3000", "--parse-requests", "0",
           "--library", "synthetic", "--patterns", "200"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["world_size"] == 8 and d["config"]["parallelism"] == "dp8"
    assert len(d["ms_per_step_per_rank"]) == 8 and d["ms_per_step"] == max(d["ms_per_step_per_rank"])
    assert d["config"]["global_batch"] == 8 * d["config"]["lines_per_gpu"]
    assert len(d["per_rank"]) == 8 and all("numa_node" in x for x in d["per_rank"])


def test_bench_single_rank_parse_over_http(tmp_path):
    """--gpus 1 --backend gloo on CPU: a process group at world size 1 (collectives still run) and
    p50 measured through a real POST /parse server process next to the engine-only latency."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "1", "--warmup", "1",
           "--backend", "gloo",
           "--lines-per-gpu", "4000", "--block-lines", "4000", "--parse-requests", "2", "--patterns", "60"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["world_size"] == 1 and d["backend"] == "gloo"
    assert d["p50_parse_ms"] > 0 and d["p50_engine_ms"] > 0
    assert "HTTP" in d["parse_transport"]


def test_bench_hang_guard_reports_phases(tmp_path):
    """A rank that hangs mid-run (rank 1 stops responding at step 2) must not burn the driver's
    timeout: within the stall limit rank 0 prints ONE JSON line with status 'timeout' and every
    rank's last completed phase, and the job exits non-zero (utils/heartbeat.py). (Stall limit
    30 s: at 12 s a loaded CPU box could stall in the set-up phases before the injected hang.)"""
    import time
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "3",
           "--warmup", "1", "--lines-per-gpu", "3000", "--block-lines", "3000", "--distinct-blocks", "1",
           "--parse-requests", "0", "--library", "synthetic", "--patterns", "50", "--stall-timeout", "30"]
    env = dict(os.environ, OMP_NUM_THREADS="1", LP_FAULT_RANK="1", LP_FAULT_STEP="2", LP_FAULT_MODE="hang",
               LP_FAULT_HANG_S="600")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    t0 = time.monotonic()
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert time.monotonic() - t0 < 200
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    d = _json_line(r.stdout)
    assert d["status"] == "timeout" and d["n_gpus"] == 2 and d["value"] is None
    assert d["phases"]["1"]["phase"] == "timed 0"           # rank 1 finished timed step 0, hung in step 1
    assert d["phases"]["0"]["phase"] in ("timed 0", "timed 1")


def test_bench_result_digest_world4_equals_world1_over_the_same_log(tmp_path):
    """The node-wide DP step is exact: 4 ranks over 4 consecutive shards (halos, both collectives,
    the local sum + top-k merge) give the same global histograms and merged top-k rows as ONE rank
    over the concatenated log (bench.py tiles rank r's blocks where rank r-1's end)."""
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "1", "--warmup", "1",
            "--block-lines", "1500", "--parse-requests", "0", "--library", "synthetic", "--patterns", "120",
            "--phase-log", str(tmp_path / "phases")]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    out = {}
    for w, lines in ((4, 3000), (1, 12000)):
        r = subprocess.run(base + ["--gpus", str(w), "--lines-per-gpu", str(lines)], cwd=str(tmp_path), env=env,
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        out[w] = _json_line(r.stdout)
    assert out[4]["config"]["global_batch"] == out[1]["config"]["global_batch"] == 12000
    assert out[4]["result_digest"] and out[4]["result_digest"] == out[1]["result_digest"]
    phases = [json.loads(l)["phase"] for l in open(tmp_path / "phases.rank3.jsonl")]
    assert "process group ready" in phases and "timed 0" in phases
