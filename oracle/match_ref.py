"""numpy restatement of the evaluation matchers (TEST ORACLE; never imported by
posfeat_amd).  Pinned against tests/golden/matchers.npz, which
tests/golden/gen_golden.py writes by running the reference's own functions:

* ``mnn_matcher``             losses/preprocess_utils.py:795-803 (the same code as
                              evaluations/hpatches/evaluation.py:28-38)
* ``mutual_nn_matcher``       evaluations/aachen/matchers.py:5-14
                              (= evaluations/ETH_local_feature/custom_matcher.py:5-14)
* ``ratio_matcher``           evaluations/aachen/matchers.py:17-44
* ``mutual_nn_ratio_matcher`` evaluations/aachen/matchers.py:47-75

sim = d1 @ d2.T in float32; nearest neighbours by arg-max with the FIRST
(lowest) index winning ties; the ratio uses the top-2 similarities of a row
(value descending, index ascending) with dist = sqrt(2 - 2 sim) and
ratio = dist1 / (dist2 + 1e-8), all in float32 as torch computes them.
Matches are returned in ascending order of the first index, as the
reference's boolean-mask indexing produces them.
"""
import numpy as np


def seeded_descriptors(seed, n1, n2, dim=128, n_common=None, noise=0.05):
    """Two L2-normalised descriptor sets with ``n_common`` true correspondences
    (d2 rows are noisy copies of shuffled d1 rows, the rest random)."""
    rs = np.random.RandomState(seed)
    d1 = rs.randn(n1, dim).astype(np.float32)
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    k = min(n1, n2) // 2 if n_common is None else n_common
    src = rs.permutation(n1)[:k]
    d2 = rs.randn(n2, dim).astype(np.float32)
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    dst = rs.permutation(n2)[:k]
    d2[dst] = d1[src] + noise * rs.randn(k, dim).astype(np.float32)
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    return d1.astype(np.float32), d2.astype(np.float32)


def _top2(sim):
    """per row: (best index, best value, second value), first index wins ties"""
    i1 = np.argmax(sim, axis=1)
    v1 = sim[np.arange(sim.shape[0]), i1]
    s2 = sim.copy()
    s2[np.arange(sim.shape[0]), i1] = -np.inf
    v2 = s2.max(axis=1)
    return i1, v1, v2


def _ratio(v1, v2):
    with np.errstate(invalid="ignore"):
        d1 = np.sqrt(np.float32(2) - np.float32(2) * v1)
        d2 = np.sqrt(np.float32(2) - np.float32(2) * v2)
        return (d1 / (d2 + np.float32(1e-8))).astype(np.float32)


def _sim(d1, d2):
    return (d1.astype(np.float32) @ d2.astype(np.float32).T).astype(np.float32)


def mnn_matcher(d1, d2):
    sim = _sim(d1, d2)
    nn12 = np.argmax(sim, axis=1)
    nn21 = np.argmax(sim, axis=0)
    ids1 = np.arange(sim.shape[0])
    mask = ids1 == nn21[nn12]
    return np.stack([ids1[mask], nn12[mask]], 1)


mutual_nn_matcher = mnn_matcher


def ratio_matcher(d1, d2, ratio=0.95):
    sim = _sim(d1, d2)
    nn12, a1, b1 = _top2(sim)
    nn21, a2, b2 = _top2(sim.T)
    r12, r21 = _ratio(a1, b1), _ratio(a2, b2)
    ids1 = np.arange(sim.shape[0])
    with np.errstate(invalid="ignore"):
        mask = (r12 <= ratio) & (r21[nn12] <= ratio)
    return np.stack([ids1[mask], nn12[mask]], 1)


def mutual_nn_ratio_matcher(d1, d2, ratio=0.95):
    sim = _sim(d1, d2)
    nn12, a1, b1 = _top2(sim)
    nn21, a2, b2 = _top2(sim.T)
    r12, r21 = _ratio(a1, b1), _ratio(a2, b2)
    ids1 = np.arange(sim.shape[0])
    with np.errstate(invalid="ignore"):
        mask = (ids1 == nn21[nn12]) & (r12 <= ratio) & (r21[nn12] <= ratio)
    return np.stack([ids1[mask], nn12[mask]], 1)
