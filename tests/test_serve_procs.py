"""Node-scale serving over processes (serve/procs.py, csrc/runtime/proc_shared.cpp): arrival tickets
and cross-process turns in shared memory, ONE frequency window in host shared memory used by every
serving process (SharedFrequencyState over N.SharedWindow; GPU workers reach it through the native
request runner's host-window section), and the supervisor + SO_REUSEPORT workers end to end: serial
requests over fresh connections give exactly the responses of the sequential reference (golden
model, one frequency tracker) -- FrequencyTrackingService.java:25 one window for every request,
ScoringService.java:84-88 -- also across a worker's death and restart."""
import http.client
import json
import multiprocessing as mp
import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import yaml

from log_parser_amd import golden
from log_parser_amd.frequency import FrequencyState, SharedFrequencyState
from log_parser_amd.native import N
from log_parser_amd.utils.config import ScoringParams
from log_parser_amd.utils.launch import free_port
from log_parser_amd.utils.synth import make_library, make_log

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _name(tag):
    return f"/lp-test-{tag}-{os.getpid()}-{time.monotonic_ns() % 10**9}"


def _turn_worker(name, n_batches, out_q):
    sh = N.ProcShared(name, False)
    got = []
    for _ in range(n_batches):
        s = sh.take()
        sh.host.wait(s)
        got.append(s)
        time.sleep(0.001)
        sh.host.done(s)
    out_q.put(got)


def test_tickets_and_turn_order_across_processes():
    """Tickets are unique across processes, and every window section starts only after all
    earlier tickets finished theirs (checked through the turn's own `next`)."""
    name = _name("turn")
    sh = N.ProcShared(name, True, 3)
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_turn_worker, args=(name, 40, q)) for _ in range(3)]
        for p in ps:
            p.start()
        got = [q.get(timeout=120) for _ in ps]
        for p in ps:
            p.join(timeout=60)
            assert p.exitcode == 0
        allt = sorted(x for g in got for x in g)
        assert allt == list(range(120))
        assert sh.host.next == 120 and sh.ticket == 120
    finally:
        N.ProcShared.unlink(name, 0)


def _die_holding(name):
    sh = N.ProcShared(name, False)
    sh.take()               # ticket 0, never released
    os._exit(3)


def test_dead_ticket_holder_is_released():
    name = _name("dead")
    sh = N.ProcShared(name, True, 2)
    try:
        p = mp.get_context("spawn").Process(target=_die_holding, args=(name,))
        p.start()
        p.join(timeout=60)
        assert p.exitcode == 3
        s = sh.take()
        t0 = time.monotonic()
        sh.dev.wait(s)                       # released after its holder is found dead (~1 s)
        assert time.monotonic() - t0 < 10 and sh.released_dead == 1
        sh.dev.done(s)
        assert sh.dev.next == 2
    finally:
        N.ProcShared.unlink(name, 0)


def _window_worker(name, ids, plan, out_q):
    sh = N.ProcShared(name, False)
    while not sh.up(0):
        time.sleep(0.01)
    fs = SharedFrequencyState(ids, 1, sh, create=False)
    res = []
    for seq, counts, now in plan:
        while sh.ticket < seq:           # draw exactly the ticket of this plan entry
            time.sleep(0.0005)
        assert sh.take() == seq
        sh.host.wait(seq)
        sh.dev.wait(seq)
        res.append((seq, fs.carry_tensor(now).numpy()[:len(ids)].tolist()))
        fs.record_tensor(torch.tensor(counts, dtype=torch.int64), now)
        sh.host.done(seq)
        sh.dev.done(seq)
    out_q.put(res)


def test_shared_window_across_processes_matches_one_window():
    """Two processes record into and read from ONE window (host shared memory), interleaved by
    ticket, with a small ring that has to grow (new generation, re-mapped by the other process):
    every carry equals a single-process FrequencyState fed in ticket order."""
    name = _name("win")
    sh = N.ProcShared(name, True, 2)
    ids = [f"k{i}" for i in range(7)]
    try:
        own = SharedFrequencyState(ids, 1, sh, create=True, capacity=16)
        sh.mark_up(0, os.getpid())
        rng = np.random.default_rng(5)
        b = sh.ticket                             # (creating the window took one ticket)
        plan = [(b + s, rng.integers(0, 3, len(ids)).tolist(), 1000.0 + 400.0 * s) for s in range(24)]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=_window_worker, args=(name, ids, [x for x in plan if x[0] % 2 == 1], q))
        p.start()
        mine = []
        for seq, counts, now in (x for x in plan if x[0] % 2 == 0):
            while sh.ticket < seq:
                time.sleep(0.0005)
            assert sh.take() == seq
            sh.host.wait(seq)
            sh.dev.wait(seq)
            mine.append((seq, own.carry_tensor(now).numpy()[:len(ids)].tolist()))
            own.record_tensor(torch.tensor(counts, dtype=torch.int64), now)
            sh.host.done(seq)
            sh.dev.done(seq)
        theirs = q.get(timeout=120)
        p.join(timeout=60)
        assert p.exitcode == 0
        got = dict(mine + theirs)
        clock = [0.0]
        fs = FrequencyState(1, clock=lambda: clock[0])
        for seq, counts, now in plan:
            clock[0] = now
            assert got[seq] == fs.carry(ids).tolist(), seq
            fs.record_counts(ids, counts, now)
        assert int(sh.generation) > 1             # the ring grew while shared
        clock[0] = own.clock()
        assert own.statistics() == fs.statistics()
    finally:
        N.ProcShared.unlink(name, int(sh.generation))


def _die_in_growth(name):
    """What a worker leaves behind when it dies inside SharedWindow::ensure_room after creating the
    next generation's block (shm_open O_EXCL + ftruncate) and before publishing it."""
    sh = N.ProcShared(name, False)
    fd = os.open(f"/dev/shm{name}.w{int(sh.generation) + 1}", os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
    os.ftruncate(fd, 1 << 16)
    os.close(fd)
    os._exit(5)


def test_window_grows_past_a_dead_workers_orphan_block_and_huge_counts():
    """A worker killed between creating and publishing a generation must not block later growth
    (the orphan block is replaced), the supervisor's unlink removes blocks past the published
    generation, and a per-key batch count above 2^31 is split over int32 ring records so that
    eviction takes back exactly what was added."""
    name = _name("orph")
    sh = N.ProcShared(name, True, 2)
    ids = ["a", "b", "c"]
    try:
        own = SharedFrequencyState(ids, 1, sh, create=True, capacity=6)
        p = mp.get_context("spawn").Process(target=_die_in_growth, args=(name,))
        p.start()
        p.join(timeout=60)
        assert p.exitcode == 5 and os.path.exists(f"/dev/shm{name}.w2")
        g0 = int(sh.generation)
        for s in range(8):                                      # 8 x 3 records through a 6-slot ring
            seq = sh.take()
            sh.host.wait(seq)
            sh.dev.wait(seq)
            own.carry_tensor(1000.0 + s)
            own.record_tensor(torch.tensor([1, 2, s], dtype=torch.int64), 1000.0 + s)
            sh.host.done(seq)
            sh.dev.done(seq)
        assert int(sh.generation) > g0
        assert own.tot.tolist() == [8, 16, sum(range(8))]
        big = 3 * (1 << 31) + 5
        own.record_tensor(torch.tensor([big, 0, 1], dtype=torch.int64), 2000.0)
        assert own.tot.tolist() == [8 + big, 16, sum(range(8)) + 1]
        assert own.carry_tensor(2000.0 + 7200.0).tolist() == [0, 0, 0]     # everything evicted, exactly
        # an orphan past the published generation is removed by the supervisor's unlink
        g = int(sh.generation)
        fd = os.open(f"/dev/shm{name}.w{g + 1}", os.O_CREAT | os.O_RDWR, 0o600)
        os.close(fd)
    finally:
        N.ProcShared.unlink(name, int(sh.generation))
    assert not [f for f in os.listdir("/dev/shm") if f.startswith(name.lstrip("/"))]


def _post(port, body):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
    try:
        c.request("POST", "/parse", body=body, headers={"content-type": "application/json"})
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def _get(port, path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    try:
        c.request("GET", path)
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def test_two_serving_processes_equal_serial_reference(tmp_path):
    """The supervisor starts 2 workers on one port (SO_REUSEPORT); 24 requests sent one after
    another, each on a fresh connection (the kernel spreads them over both processes), get the
    golden model's responses with ONE frequency tracker -- the penalty of every request sees the
    counts recorded by the other process."""
    _serve(tmp_path, "cpu", 2)


def test_four_serving_processes_equal_serial_reference(tmp_path):
    _serve(tmp_path, "cpu", 4, n_req=28)


@pytest.mark.gpu
@pytest.mark.parametrize("nproc", [2, 4])
def test_gpu_serving_processes_equal_serial_reference(tmp_path, nproc):
    """The same with every worker on cuda:0 (the one-GPU rehearsal of one process per GPU): the
    window is host shared memory, each worker's native request runner evicts / reads the carry /
    records it inside its window section (ticket drawn after its matching) -- /ready reports the
    native runner in EVERY worker, and the responses equal the golden model's (rtol 1e-12)."""
    _serve(tmp_path, "cuda:0", nproc, n_req=40)


def test_worker_death_survivors_serve_and_restart(tmp_path):
    """A worker killed with SIGKILL: the survivors keep answering (golden responses, the window
    intact), the supervisor restarts the dead worker on the same device, the new process attaches
    to the existing window and serves too."""
    _serve(tmp_path, "cpu", 2, n_req=16, kill_after=6)


def _ready_pids(port, want, deadline_s=240, sup=None, log=None):
    pids = set()
    deadline = time.monotonic() + deadline_s
    while len(pids) < want:                    # every worker answers (each reports its pid)
        if sup is not None:
            assert sup.poll() is None, log.read_text()[-3000:] if log else ""
        assert time.monotonic() < deadline, "workers did not come up"
        try:
            st, body = _get(port, "/ready")
            if st == 200:
                pids.add(json.loads(body)["worker"]["pid"])
        except OSError:
            time.sleep(0.2)
    return pids


def _serve(tmp_path, device, nproc, n_req=24, extra=(), kill_after=None):
    sets, trig = make_library(20, seed=91)
    for i, s in enumerate(sets):
        (tmp_path / f"lib{i}.yaml").write_text(yaml.safe_dump(s.model_dump(by_alias=True, exclude_none=True)))
    port = free_port()
    cmd = [sys.executable, "-m", "log_parser_amd.serve", f"-Dpattern.directory={tmp_path}", f"-Dengine.device={device}",
           f"-Dserver.processes={nproc}", f"-Dserver.port={port}", "-Dserver.host=127.0.0.1",
           "-Dscoring.frequency.threshold=1.0", "-Dserver.numa-bind=false"] + list(extra)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    logf = open(tmp_path / "serve.log", "wb")
    sup = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=logf)
    try:
        pids = _ready_pids(port, nproc, sup=sup, log=tmp_path / "serve.log")
        params = ScoringParams(freq_threshold=1.0)
        tracker = golden.FrequencyTracker(params)
        for i in range(n_req):
            if kill_after is not None and i == kill_after:
                victim = sorted(pids)[-1]
                os.kill(victim, signal.SIGKILL)        # idle: it holds no ticket
                time.sleep(0.5)
            logs = make_log(150 + 31 * (i % 4), trig, seed=700 + i, hit_rate=0.12)
            st, out = _post(port, json.dumps({"pod": {"metadata": {"name": f"p{i}"}}, "logs": logs}).encode())
            assert st == 200
            o, g = json.loads(out), golden.analyze(logs, sets, params, tracker)
            assert o["summary"] == g["summary"], i
            assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
                   [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]], i
            assert [e["score"] for e in o["events"]] == pytest.approx([e["score"] for e in g["events"]], rel=1e-12)
        if kill_after is not None:             # the dead worker was restarted and attached to the window
            now = _ready_pids(port, nproc, sup=sup, log=tmp_path / "serve.log")
            assert victim not in now
            assert b"restarting it" in (tmp_path / "serve.log").read_bytes()
        if device != "cpu":                 # every worker serves through the native runner (host window)
            seen = {}
            for _ in range(20 * nproc):
                r = json.loads(_get(port, "/ready")[1])
                seen[r["worker"]["pid"]] = r["nativeRunner"]
            assert len(seen) == nproc and all(seen.values()), seen
        # the admin API reads the one window from either process
        stats = [json.loads(_get(port, "/admin/frequency")[1]) for _ in range(4)]
        assert all(s == stats[0] for s in stats) and sum(stats[0].values()) > 0
    finally:
        sup.send_signal(signal.SIGTERM)
        try:
            sup.wait(timeout=60)
        except subprocess.TimeoutExpired:
            sup.kill()
            sup.wait()
        logf.close()


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_engines_over_host_window_equal_golden(dev):
    """Two GPU engines (as two serving processes would) over ONE host shared window: every batch
    runs through the native request runner's host-window section -- ticket after the matching,
    host eviction + pinned carry, score kernel, host record -- and the responses equal the golden
    model with one tracker (rtol 1e-12), alternating engines batch by batch. On CPU: the Python
    path's late ticket over the same window."""
    from log_parser_amd.engine import Engine, ProcessWindowTurn
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.utils.config import Config
    name = _name("hw")
    sh = N.ProcShared(name, True, 2)
    try:
        sets, trig = make_library(30, seed=93, sequence_rate=0.6)
        params = ScoringParams(freq_threshold=1.0)
        lib = CompiledLibrary(sets, params)
        fs = [SharedFrequencyState(lib.freq_ids, 1, sh, create=True)]
        fs.append(SharedFrequencyState(lib.freq_ids, 1, sh, create=False))
        cfg = Config.load(overrides={"engine.device": dev})
        engs = [Engine(lib, cfg, device=torch.device(dev), freq=f) for f in fs]
        turn = ProcessWindowTurn(sh)
        tracker = golden.FrequencyTracker(params)
        s0 = int(sh.sections)
        for i in range(14):
            docs = [make_log(120 + 17 * (i % 3), trig, seed=900 + i, hit_rate=0.15)]
            if i % 5 == 4:
                docs.append(make_log(90, trig, seed=950 + i, hit_rate=0.2))      # a 2-request batch
            outs = engs[i % 2].analyze_batch_json(docs, turn, None)
            for o, d in zip(outs, docs):
                o, g = json.loads(o), golden.analyze(d, sets, params, tracker)
                assert [(e["lineNumber"], e["matchedPattern"]["id"]) for e in o["events"]] == \
                       [(e["lineNumber"], e["matchedPattern"]["id"]) for e in g["events"]], i
                np.testing.assert_allclose([e["score"] for e in o["events"]], [e["score"] for e in g["events"]],
                                           rtol=1e-12)
        if dev != "cpu":
            assert all(e._runner not in (None, False) for e in engs)
        assert int(sh.sections) - s0 == 14 or dev == "cpu"
        assert fs[1].statistics() == {k: v for k, v in tracker.statistics().items() if v}
    finally:
        N.ProcShared.unlink(name, int(sh.generation))
