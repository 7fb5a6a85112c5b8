"""GPU parity of the evaluation matchers (posfeat_amd.matchers, match.hip)
against the reference's own outputs (tests/golden/matchers.npz) and the
numpy oracle.  Index-exact; a differing match is only accepted when the
comparison that decides it is a near-tie of the float64 similarities
(|margin| < 1e-5: the GPU's fp32 fmaf-chain dot products and the CPU
reference's BLAS order differ by ~1e-7)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import match_ref as mr

pytestmark = pytest.mark.gpu

CASES = [(11, 1000, 1200), (12, 2048, 2048), (13, 500, 300), (14, 4096, 3000)]
TIE = 1e-5


def _explained(d1, d2, got, ref, ratio=None):
    """rows i whose match differs and whose deciding comparison is not a near-tie"""
    s = d1.astype(np.float64) @ d2.astype(np.float64).T
    a, b = {tuple(m) for m in got.tolist()}, {tuple(m) for m in ref.tolist()}
    bad = []
    for i, _ in sorted(a ^ b):
        row = np.sort(s[i])[::-1]
        j = int(np.argmax(s[i]))
        col = np.sort(s[:, j])[::-1]
        margins = [row[0] - row[1], col[0] - col[1]]
        if ratio is not None:
            q = lambda v: np.sqrt(max(2 - 2 * v[0], 0)) / (np.sqrt(max(2 - 2 * v[1], 0)) + 1e-8)
            margins += [abs(q(row) - ratio), abs(q(col) - ratio)]
        if min(margins) >= TIE:
            bad.append(i)
    return bad


@pytest.mark.parametrize("seed,n1,n2", CASES)
def test_matchers_vs_reference(gpu, seed, n1, n2):
    from posfeat_amd import matchers as M
    d = np.load(os.path.join(GOLDEN, "matchers.npz"))
    tag = "m%d" % seed
    d1, d2 = mr.seeded_descriptors(seed, n1, n2)
    t1, t2 = torch.from_numpy(d1).to(gpu), torch.from_numpy(d2).to(gpu)
    checks = [(M.mnn_matcher(t1, t2), d[tag + "_mnn"], None),
              (M.mutual_nn_matcher(t1, t2), d[tag + "_eth_mutual_nn"], None)]
    for r in (0.95, 0.8):
        checks.append((M.ratio_matcher(t1, t2, ratio=r), d["%s_ratio_%g" % (tag, r)], r))
        checks.append((M.mutual_nn_ratio_matcher(t1, t2, ratio=r),
                       d["%s_mnn_ratio_%g" % (tag, r)], r))
    for got, ref, r in checks:
        assert got.dtype == np.int64 and got.ndim == 2 and got.shape[1] == 2
        if not np.array_equal(got, ref):
            assert _explained(d1, d2, got, ref, r) == []
        assert np.all(np.diff(got[:, 0]) > 0)          # ascending first index


def test_matchers_hpatches_scale_vs_oracle(gpu):
    """8192 x 8192 (configs/extract_hpatches.yaml num_pts) and a ragged
    20480 x 7000 pair (Aachen num_pts) against the numpy oracle."""
    from posfeat_amd import matchers as M
    for seed, n1, n2 in ((21, 8192, 8192), (22, 20480, 7000)):
        d1, d2 = mr.seeded_descriptors(seed, n1, n2)
        t1, t2 = torch.from_numpy(d1).to(gpu), torch.from_numpy(d2).to(gpu)
        for fn, r in ((M.mnn_matcher, None), (M.mutual_nn_ratio_matcher, 0.9)):
            got = fn(t1, t2) if r is None else fn(t1, t2, ratio=r)
            ref = (mr.mnn_matcher(d1, d2) if r is None
                   else mr.mutual_nn_ratio_matcher(d1, d2, r))
            if not np.array_equal(got, ref):
                assert _explained(d1, d2, got, ref, r) == []


def test_matcher_tie_rule_and_edge_cases(gpu):
    """Exact duplicate descriptors: the first index wins; empty inputs; the
    drop-in in losses.preprocess_utils; the loud failure for other dims."""
    from posfeat_amd import matchers as M
    from posfeat_amd.losses import preprocess_utils as pu
    rs = np.random.RandomState(5)
    d1 = rs.randn(300, 128).astype(np.float32)
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    d2 = np.concatenate([d1[:100], d1[:100], d1[100:]], 0)   # d2 rows j and j+100 tie
    got = M.mnn_matcher(torch.from_numpy(d1).to(gpu), torch.from_numpy(d2).to(gpu))
    ref = mr.mnn_matcher(d1, d2)
    np.testing.assert_array_equal(got, ref)
    assert got[:100, 1].tolist() == list(range(100))         # first occurrence
    np.testing.assert_array_equal(pu.mnn_matcher(torch.from_numpy(d1).to(gpu),
                                                 torch.from_numpy(d2).to(gpu)), ref)
    assert M.mnn_matcher(np.zeros((0, 128), np.float32), d2).shape == (0, 2)
    # one descriptor on a side: the reference's topk(k=2) raises, and so do we
    for f in (M.ratio_matcher, M.mutual_nn_ratio_matcher):
        for a, b in ((d1[:1], d2), (d1, d2[:1])):
            with pytest.raises(RuntimeError):
                f(a, b)
    assert M.mnn_matcher(d1[:1], d2).shape == (1, 2)
    with pytest.raises(NotImplementedError):
        M.mnn_matcher(np.zeros((4, 64), np.float32), np.zeros((4, 64), np.float32))
