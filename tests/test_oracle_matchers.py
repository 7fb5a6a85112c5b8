"""Pin the matcher oracle (oracle/match_ref.py) against the reference's own
matchers run on seeded descriptor sets (tests/golden/matchers.npz, written by
tests/golden/gen_golden.py from losses/preprocess_utils.py:795-803,
evaluations/aachen/matchers.py and evaluations/ETH_local_feature/
custom_matcher.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import match_ref as mr

CASES = [(11, 1000, 1200), (12, 2048, 2048), (13, 500, 300), (14, 4096, 3000)]


@pytest.mark.parametrize("seed,n1,n2", CASES)
def test_matcher_oracle_vs_reference(seed, n1, n2):
    d = np.load(os.path.join(GOLDEN, "matchers.npz"))
    tag = "m%d" % seed
    assert tuple(d[tag + "_shape"]) == (n1, n2)
    d1, d2 = mr.seeded_descriptors(seed, n1, n2)
    np.testing.assert_array_equal(mr.mnn_matcher(d1, d2), d[tag + "_mnn"])
    np.testing.assert_array_equal(mr.mutual_nn_matcher(d1, d2), d[tag + "_mutual_nn"])
    np.testing.assert_array_equal(mr.mutual_nn_matcher(d1, d2), d[tag + "_eth_mutual_nn"])
    for r in (0.95, 0.8):
        np.testing.assert_array_equal(mr.ratio_matcher(d1, d2, r), d["%s_ratio_%g" % (tag, r)])
        np.testing.assert_array_equal(mr.mutual_nn_ratio_matcher(d1, d2, r),
                                      d["%s_mnn_ratio_%g" % (tag, r)])


def test_matcher_oracle_tie_rule():
    """Stated tie rule: the first (lowest) index wins an arg-max tie."""
    d1 = np.eye(4, 8, dtype=np.float32)
    d2 = np.concatenate([d1[:1], d1[:1], d1[1:]], 0)   # rows 0 and 1 of d2 tie for d1[0]
    m = mr.mnn_matcher(d1, d2)
    assert m[0].tolist() == [0, 0]
