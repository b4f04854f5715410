"""Summary + top-k kernel chain (csrc/kernels/summarize.hip) and the streaming re-score kernel.

Reference for both: plain numpy/PyTorch fp64 of the same op -- a full lexicographic sort by
(score desc, global line asc, pattern asc) and bincounts; the reference's chronological factor
(golden.chronological_factor, ScoringService.java:125-151) in the product order of
ScoringService.java:102-109. Ties are deliberate (few distinct scores) so the order is pinned.
"""
import numpy as np
import pytest
import torch

from log_parser_amd.ops import kernels as K


def _events(n, npat, nsev, seed, line64=False):
    rng = np.random.default_rng(seed)
    score = rng.choice(np.array([0.5, 1.25, 3.0, 7.5, 7.5000000000000009]), size=n)
    line = np.sort(rng.integers(0, max(1, n // 2), size=n)).astype(np.int64 if line64 else np.int32)
    pat = rng.integers(0, npat, size=n).astype(np.int32)
    sev_index = rng.integers(0, nsev, size=npat).astype(np.int32)
    return score, line, pat, sev_index


def _ref(score, line, pat, add, k, sev_index, npat, nsev):
    gl = line.astype(np.int64) + add
    order = np.lexsort((pat, gl, -score))[:k]
    rows = np.full((k, 3), -1.0)
    rows[:, 0] = -np.inf
    m = order.size
    rows[:m, 0] = score[order]
    rows[:m, 1] = gl[order]
    rows[:m, 2] = pat[order]
    ph = np.bincount(pat, minlength=npat)
    sh = np.bincount(sev_index[pat], minlength=nsev) if pat.size else np.zeros(nsev, np.int64)
    return rows, ph, sh


def _run(dev, score, line, pat, sev_index, k, npat, nsev, add):
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    la = T(np.array([add], np.int64)) if add else None
    rows, ph, sh, packed = K.summarize(T(score), T(pat), T(line), k, T(sev_index), npat, nsev, line_add=la,
                                      pack_events=True)
    pk = packed.cpu().numpy()
    n = score.size
    np.testing.assert_array_equal(pk[:8 * n].view(np.int64), line.astype(np.int64) + add)
    np.testing.assert_array_equal(pk[8 * n:16 * n].view(np.float64), score)
    np.testing.assert_array_equal(pk[16 * n:].view(np.int32), pat)
    return rows.cpu().numpy(), ph.cpu().numpy(), sh.cpu().numpy()


CASES = [(0, 5), (1, 5), (7, 5), (2047, 100), (2048, 100), (2049, 1), (50_000, 100), (50_000, 1024),
         (300_000, 37), (50_000, 256), (50_000, 257)]     # 256 / 257: the 1024-row / 4096-row chunk variants


@pytest.mark.parametrize("n,k", CASES)
def test_summarize_cpu_matches_reference(n, k):
    score, line, pat, sev_index = _events(n, 61, 4, seed=n + k)
    got = _run("cpu", score, line, pat, sev_index, k, 61, 4, 1000)
    ref = _ref(score, line, pat, 1000, k, sev_index, 61, 4)
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(got[2], ref[2])


def test_topk_rows_merge_cpu():
    rng = np.random.default_rng(3)
    parts = []
    for r in range(5):
        score, line, pat, sev = _events(3000, 17, 3, seed=r, line64=True)
        rows, _, _ = _run("cpu", score, line + r * 10_000, pat, sev, 50, 17, 3, 0)
        parts.append(rows)
    allrows = np.concatenate(parts)
    rng.shuffle(allrows)
    got = K.topk_rows(torch.from_numpy(allrows), 50).numpy()
    fin = allrows[np.isfinite(allrows[:, 0])]
    order = np.lexsort((fin[:, 2], fin[:, 1], -fin[:, 0]))[:50]
    np.testing.assert_array_equal(got, fin[order])


def test_rescore_matches_reference_order():
    from log_parser_amd.engine import Engine
    from log_parser_amd.golden import chronological_factor
    from log_parser_amd.utils.config import ScoringParams
    p = ScoringParams()
    sp = Engine.score_param_tuple(p)
    rng = np.random.default_rng(7)
    n, N = 4000, 12345
    gl = np.sort(rng.integers(0, N, size=n)).astype(np.int64)
    fac = rng.uniform(0.1, 3.0, size=(n, 7))
    fac[:, 6] = rng.uniform(0, 0.5, size=n)
    got = K.rescore(torch.from_numpy(gl), torch.from_numpy(fac), N, sp).numpy()
    ref = np.array([fac[i, 0] * fac[i, 1] * chronological_factor(int(gl[i]), N, p) * fac[i, 3] * fac[i, 4] * fac[i, 5]
                    * (1.0 - fac[i, 6]) for i in range(n)])
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("select", [False, True])
@pytest.mark.parametrize("n,k", CASES)
def test_summarize_gpu_equals_cpu(gpu_device, n, k, select):
    """Both device top-k paths: the chunk-sort levels (default) and the threshold selection
    (summarize.hip k_sel_*, N.set_summ_select)."""
    from log_parser_amd.native import N
    score, line, pat, sev_index = _events(n, 61, 4, seed=n + k)
    N.set_summ_select(select)
    try:
        got = _run(gpu_device, score, line, pat, sev_index, k, 61, 4, 77)
    finally:
        N.set_summ_select(False)
    ref = _ref(score, line, pat, 77, k, sev_index, 61, 4)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


@pytest.mark.gpu
def test_summarize_gpu_large_multilevel(gpu_device):
    """12M events: level 0 has 5860 blocks, two more merge levels."""
    n, k = 12_000_000, 100
    score, line, pat, sev_index = _events(n, 4000, 5, seed=11)
    got = _run(gpu_device, score, line, pat, sev_index, k, 4000, 5, 0)
    ref = _ref(score, line, pat, 0, k, sev_index, 4000, 5)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


@pytest.mark.gpu
def test_rescore_gpu_equals_cpu(gpu_device):
    from log_parser_amd.engine import Engine
    from log_parser_amd.utils.config import ScoringParams
    sp = Engine.score_param_tuple(ScoringParams())
    rng = np.random.default_rng(8)
    n, N = 100_000, 1_000_003
    gl = torch.from_numpy(np.sort(rng.integers(0, N, size=n)).astype(np.int64))
    fac = torch.from_numpy(rng.uniform(0.1, 3.0, size=(n, 7)))
    a = K.rescore(gl, fac, N, sp)
    b = K.rescore(gl.to(gpu_device), fac.to(gpu_device), N, sp).cpu()
    assert torch.equal(a, b)
