"""Line-sharded data parallelism (parallel/dp.py) on CPU with gloo, world_size 2, 3, 4 and 8
(the driver's scaling run launches 8 ranks: the 8-rank halo / carry / top-k paths are rehearsed
here on CPU).

The sharded pipeline (halos + packed all_gather carries + all_reduce histograms + top-k gather)
must reproduce the single-process run event for event and score for score, over consecutive
steps (the persistent frequency state and the cross-shard backward sequence chain included).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from log_parser_amd.engine import Engine, Segments
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.ops import kernels as K
from log_parser_amd.parallel.dp import ShardedAnalyzer, shard_bounds
from log_parser_amd.utils.config import Config, ScoringParams
from log_parser_amd.utils.synth import make_library, make_log

STEPS = 2


def _setup():
    sets, trig = make_library(40, seed=31, sequence_rate=0.8)
    lib = CompiledLibrary(sets, ScoringParams())
    logs = make_log(3000, trig, seed=32, hit_rate=0.08, crlf_rate=0.1)
    return lib, logs.encode()


def _text(data: bytes):
    t = torch.zeros(K.padded_len(len(data)), dtype=torch.uint8)
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    return t


def _reference():
    lib, data = _setup()
    eng = Engine(lib, Config.load(overrides={"engine.device": "cpu"}), device=torch.device("cpu"))
    t = _text(data)
    ls, ll = K.split_lines(t, len(data))
    outs = []
    for _ in range(STEPS):
        res = eng.run(t, len(data), ls, ll, Segments.single(ls.numel(), t.device), eng.freq_carry())
        eng.commit_frequency(res.freq_counts)
        outs.append((res.ev_line.numpy().astype(np.int64), res.ev_pat.numpy(), res.score.numpy(), ls.numel()))
    return outs


def _worker(rank, world, port, q, dev="cpu", tiny_rank=-1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lib, data = _setup()
        device = torch.device(dev)
        eng = Engine(lib, Config.load(overrides={"engine.device": dev}), device=device)
        full = _text(data).to(device)
        gls, gll = K.split_lines(full, len(data))
        L = gls.numel()
        lo, hi, hl, hr = shard_bounds(L, world, rank, lib.halo)
        a, b = lo - hl, hi + hr
        base = int(gls[a])
        end = int(gls[b]) if b < L else len(data)
        shard = data[base:end]
        t = _text(shard).to(device)
        ls = (gls[a:b] - base).contiguous()
        ll = gll[a:b].contiguous()
        sa = ShardedAnalyzer(eng)
        if rank == tiny_rank:              # this rank's buffers overflow on the first step
            eng.arena.rate = {k: 1e-6 for k in eng.arena.rate}
        res = []
        for _ in range(STEPS):
            out = sa.step(t, len(shard), ls, ll, hl, hr, topk=5)
            r = out.result
            gl = (r.ev_line.cpu().numpy().astype(np.int64) - hl + out.own_start)
            res.append((gl, r.ev_pat.cpu().numpy(), r.score.cpu().numpy(), out.total_lines,
                        None if out.topk_score is None else out.topk_score.cpu().numpy()))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_sharded(world, dev, tiny_rank=-1):
    ref = _reference()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, dev, tiny_rank)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for s in range(STEPS):
        lines = np.concatenate([got[r][s][0] for r in range(world)])
        pats = np.concatenate([got[r][s][1] for r in range(world)])
        scores = np.concatenate([got[r][s][2] for r in range(world)])
        rl, rp, rs, n_lines = ref[s]
        for r in range(world):                # C1: every rank sees the global line count N
            assert got[r][s][3] == n_lines
        np.testing.assert_array_equal(lines, rl)
        np.testing.assert_array_equal(pats, rp)
        np.testing.assert_allclose(scores, rs, rtol=1e-13, atol=0)
        top = np.sort(rs)[::-1][:5]
        np.testing.assert_allclose(got[0][s][4], top, rtol=1e-13)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_equals_single(world):
    _run_sharded(world, "cpu")


@pytest.mark.gpu
def test_sharded_equals_single_gpu_ranks(gpu_device):
    """2 ranks on the one GPU of the test box: the gfx950 pipeline of every rank + the packed
    carries / histograms / top-k collectives (host-staged gloo here; RCCL on a multi-GPU node)
    must reproduce the single-process CPU reference event for event."""
    _run_sharded(2, "cuda:0")


@pytest.mark.gpu
def test_sharded_one_rank_overflow_gpu_ranks(gpu_device):
    """GPU steps read no counts until their end: rank 1 starts with capacities far too small, its
    overflow flag travels in collective 1, BOTH ranks veto the frequency record and re-run the
    step, and every step still equals the single-process reference (window recorded once)."""
    _run_sharded(2, "cuda:0", tiny_rank=1)


def _worker_p2p(rank, world, port, q, dev="cpu"):
    """Each rank holds ONLY its own lines; halos come from the neighbours over send/recv (C2)."""
    from log_parser_amd.parallel.dp import assemble_shard, exchange_halos, halo_bytes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lib, data = _setup()
        device = torch.device(dev)
        eng = Engine(lib, Config.load(overrides={"engine.device": dev}), device=device)
        full = _text(data).to(device)
        gls, gll = K.split_lines(full, len(data))
        L = gls.numel()
        lo, hi, _, _ = shard_bounds(L, world, rank, lib.halo)
        base = int(gls[lo])
        end = int(gls[hi]) if hi < L else len(data)
        own_b = data[base:end]
        head, tail = halo_bytes(own_b, lib.halo)
        own = _text(own_b).to(device)
        left, right = exchange_halos(own, len(own_b), head, tail)
        t, n, ls, ll, hl, hr = assemble_shard(own, len(own_b), left, right)
        sa = ShardedAnalyzer(eng)
        res = []
        for _ in range(STEPS):
            out = sa.step(t, n, ls, ll, hl, hr, topk=5)
            r = out.result
            gl = (r.ev_line.cpu().numpy().astype(np.int64) - hl + out.own_start)
            res.append((gl, r.ev_pat.cpu().numpy(), r.score.cpu().numpy(), out.total_lines,
                        None if out.topk_score is None else out.topk_score.cpu().numpy()))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_p2p_halo_exchange_equals_single(world):
    _run_p2p(world, "cpu")


@pytest.mark.gpu
def test_p2p_halo_exchange_gpu_ranks(gpu_device):
    _run_p2p(2, "cuda:0")


def _run_p2p(world, dev):
    ref = _reference()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_p2p, args=(r, world, port, q, dev)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for s in range(STEPS):
        rl, rp, rs, n_lines = ref[s]
        assert all(got[r][s][3] == n_lines for r in range(world))
        np.testing.assert_array_equal(np.concatenate([got[r][s][0] for r in range(world)]), rl)
        np.testing.assert_array_equal(np.concatenate([got[r][s][1] for r in range(world)]), rp)
        np.testing.assert_allclose(np.concatenate([got[r][s][2] for r in range(world)]), rs, rtol=1e-13, atol=0)


def _worker_nccl1(port, q):
    """One rank, RCCL (nccl backend) at world size 1 on the test GPU: the device-tensor in-place
    all-gathers the 8-GPU run uses, against the single-process engine."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        lib, data = _setup()
        eng = Engine(lib, Config.load(overrides={"engine.device": "cuda:0"}), device=dev)
        t = _text(data).to(dev)
        ls, ll = K.split_lines(t, len(data))
        sa = ShardedAnalyzer(eng)
        res = []
        for _ in range(STEPS):
            out = sa.step(t, len(data), ls, ll, 0, 0, topk=5)
            r = out.result
            res.append((r.ev_line.cpu().numpy().astype(np.int64), r.ev_pat.cpu().numpy(), r.score.cpu().numpy(),
                        out.total_lines, out.topk_score.cpu().numpy(), out.topk_line.cpu().numpy(),
                        out.pattern_counts.cpu().numpy()))
        q.put(("ok", res, dist.get_backend()))
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_nccl_world1_equals_engine(gpu_device):
    """ShardedAnalyzer under RCCL at world 1 == Engine.run on the whole log, top-k included."""
    ref = _reference()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl1, args=(_free_port(), q))
    p.start()
    status, res, backend = q.get(timeout=300)
    p.join(timeout=60)
    assert status == "ok", res
    assert backend == "nccl" and p.exitcode == 0
    for s in range(STEPS):
        rl, rp, rs, n_lines = ref[s]
        gl, gp, gs, tot, top, topl, pc = res[s]
        assert tot == n_lines
        np.testing.assert_array_equal(gl, rl)
        np.testing.assert_array_equal(gp, rp)
        np.testing.assert_allclose(gs, rs, rtol=1e-13, atol=0)
        order = np.lexsort((rl, -rs))[:5]                # score desc, line asc
        np.testing.assert_allclose(top, rs[order], rtol=1e-13)
        np.testing.assert_array_equal(topl, rl[order])
        assert pc.sum() == rl.size
