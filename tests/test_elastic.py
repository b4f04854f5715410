"""Elastic DP (parallel/elastic.py): a rank killed mid-job by fault injection must leave the
survivors producing exactly the single-process results, step for step (gloo, CPU).

Scenario: 3 ranks, 3 steps over the same log (the frequency state carries across steps), original
rank 2 exits at the start of step 1 (``LP_FAULT_RANK=2 LP_FAULT_STEP=1``). Step 0 commits on 3
ranks; step 1 aborts, the survivors roll the frequency state back, rebuild a 2-rank group and
re-run it; step 2 runs on 2 ranks.
"""
import os

import numpy as np
import pytest
import torch

from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log

STEPS = 3


def _setup():
    sets, trig = make_library(40, seed=41, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(2500, trig, seed=42, hit_rate=0.08, crlf_rate=0.1)
    return lib, logs.encode()


def _reference():
    lib, data = _setup()
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ls, ll = K.split_lines(t, len(data))
    outs = []
    for _ in range(STEPS):
        res = eng.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), eng.freq_carry())
        eng.commit_frequency(res.freq_counts)
        outs.append((res.ev_line.numpy().astype(np.int64), res.ev_pat.numpy(), res.score.numpy()))
    return outs


def _worker(rank, world, host, port, outdir, timeout_s=20.0):
    from log_parser_amd.parallel.elastic import ElasticAnalyzer, ElasticGroup, connect
    lib, data = _setup()
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    grp = ElasticGroup(connect(host, port), rank, world, backend="gloo", timeout_s=timeout_s, grace_s=3.0)
    ea = ElasticAnalyzer(eng, grp)
    rec = {}
    for s in range(STEPS):
        out = ea.step(data, topk=5)
        r = out.result
        rec[f"lines{s}"] = r.ev_line.numpy().astype(np.int64) - ea.halo_left + out.own_start
        rec[f"start{s}"] = np.array([out.own_start])
        rec[f"pat{s}"] = r.ev_pat.numpy()
        rec[f"score{s}"] = r.score.numpy()
        rec[f"world{s}"] = np.array([grp.size, grp.rank])
        if out.topk_score is not None:
            rec[f"top{s}"] = out.topk_score.numpy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **rec)
    grp.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_rank_failure_degrades_to_survivors(tmp_path, mode):
    from log_parser_amd.parallel.elastic import launch
    ref = _reference()
    env = {"LP_FAULT_RANK": "2", "LP_FAULT_STEP": "1", "LP_FAULT_MODE": mode, "LP_FAULT_HANG_S": "12"}
    codes = launch(_worker, 3, args=(str(tmp_path), 4.0 if mode == "hang" else 20.0), env=env, join_timeout=240)
    assert codes[2] == (17 if mode == "exit" else 18) and codes[0] == 0 and codes[1] == 0, codes
    got = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in (0, 1)]
    assert not (tmp_path / "rank2.npz").exists()
    for s in range(STEPS):
        assert got[0][f"world{s}"][0] == (3 if s == 0 else 2)
        rl, rp, rs = ref[s]
        if s == 0:
            continue  # rank 2's share of step 0 died with it; checked through top-k below
        lines = np.concatenate([g[f"lines{s}"] for g in got])
        pats = np.concatenate([g[f"pat{s}"] for g in got])
        scores = np.concatenate([g[f"score{s}"] for g in got])
        np.testing.assert_array_equal(lines, rl)
        np.testing.assert_array_equal(pats, rp)
        np.testing.assert_allclose(scores, rs, rtol=1e-13, atol=0)
    for s in range(STEPS):
        top = np.sort(ref[s][2])[::-1][:5]
        np.testing.assert_allclose(got[0][f"top{s}"], top, rtol=1e-13)


def test_rccl_rebuild_aborts_instead_of_destroying(monkeypatch):
    """On RCCL a rebuild must ncclCommAbort the old communicator (_abort_process_group): a
    destroy_process_group would wait for the dead peer's outstanding collectives."""
    from datetime import timedelta
    import torch.distributed as dist
    from log_parser_amd.parallel import elastic as E
    calls = []
    monkeypatch.setattr(E.ElasticGroup, "_init_pg", lambda self: calls.append("init"))
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist.distributed_c10d, "_abort_process_group", lambda group=None: calls.append("abort"))
    monkeypatch.setattr(dist, "destroy_process_group", lambda group=None: calls.append("destroy"))
    store = dist.HashStore()
    g = E.ElasticGroup(store, 0, 1, backend="nccl", timeout_s=5.0, grace_s=0.05)
    g.rebuild()
    assert calls == ["init", "abort", "init"] and g.members == [0] and g.gen == 1
    calls.clear()
    g.backend = "gloo"
    g.rebuild()
    assert calls == ["destroy", "init"]


def _abort_worker(host, port, q):
    """World-1 RCCL communicator: collective -> real _abort_process_group -> re-init -> collective,
    then an elastic analysis step on the rebuilt group."""
    import torch.distributed as dist
    from log_parser_amd.parallel.elastic import ElasticAnalyzer, ElasticGroup, connect
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        grp = ElasticGroup(connect(host, port), 0, 1, backend="nccl", timeout_s=30.0, grace_s=0.2, device=dev)
        x = torch.arange(8, dtype=torch.int64, device=dev)
        dist.all_reduce(x)
        before = x.cpu().tolist()
        grp.rebuild()                                    # ncclCommAbort, new generation, new communicator
        y = torch.full((4,), 3, dtype=torch.int64, device=dev)
        dist.all_reduce(y)
        after = y.cpu().tolist()
        lib, data = _setup()
        eng = Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
        out = ElasticAnalyzer(eng, grp).step(data, topk=5)
        q.put(("ok", before, after, grp.gen, out.result.score.cpu().numpy(), dist.get_backend()))
        grp.close()
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e), None, None, None, None))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_abort_reinit_cycle_world1(gpu_device):
    """The RCCL teardown of a rebuild runs for real (not monkeypatched): at world 1 on the test GPU
    a collective, ncclCommAbort through _abort_process_group, a new generation's communicator and
    a collective on it, then an elastic step equal to the single-process reference."""
    import multiprocessing as mp
    from datetime import timedelta
    import torch.distributed as dist
    store = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=timedelta(seconds=120))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_abort_worker, args=("127.0.0.1", store.port, q))
    p.start()
    r = q.get(timeout=240)
    p.join(timeout=60)
    assert r[0] == "ok", r[1]
    _, before, after, gen, score, backend = r
    assert before == list(range(8)) and after == [3, 3, 3, 3] and gen == 1 and backend == "nccl"
    np.testing.assert_allclose(score, _reference()[0][2], rtol=1e-13, atol=0)
