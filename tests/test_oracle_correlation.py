"""Pin the correlation oracle (oracle/correlation_ref.py) against golden
vectors from the reference's own Preprocess_Line2Window, EpipolarLoss_full
and DiskLoss (tests/golden/gen_golden.py, random draws replayed)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import correlation_ref as cr


def _inputs(tag):
    import sys
    sys.path.insert(0, GOLDEN)
    from posfeat_amd.correlation import synthetic_fundamental
    b, H, W, seed = {"s": (2, 240, 320, 3), "f": (1, 480, 640, 4)}[tag]
    rs = np.random.RandomState(seed)
    xf1 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    xf2 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    xf1 = torch.nn.functional.avg_pool2d(xf1, 3, 1, 1)
    xf2 = torch.nn.functional.avg_pool2d(xf2, 3, 1, 1)
    kp1 = torch.from_numpy(rs.rand(b, 1, H, W).astype(np.float32) * 3)
    kp2 = torch.from_numpy(rs.rand(b, 1, H, W).astype(np.float32) * 3)
    F1, F2 = synthetic_fundamental(b, H, W, seed)
    return b, H, W, xf1, xf2, kp1, kp2, torch.from_numpy(F1), torch.from_numpy(F2)


@pytest.mark.parametrize("tag", ["s", "f"])
def test_line2window_and_epipolar_loss_oracle(tag):
    d = np.load(os.path.join(GOLDEN, "correlation.npz"))
    b, H, W, xf1, xf2, kp1, kp2, F1, F2 = _inputs(tag)
    g = lambda k: torch.from_numpy(d["%s_%s" % (tag, k)])  # noqa: E731
    proc = cr.line2window(xf1, xf2, F1, F2, (H, W), (H, W), g("sel1").long(), g("sel2").long(),
                          g("rand1"), g("rand2"))
    for k, v in proc.items():
        if not torch.is_tensor(v):
            continue
        ref = d["%s_proc_%s" % (tag, k)]
        if v.dtype == torch.bool:
            np.testing.assert_array_equal(v.numpy(), ref, err_msg=k)
        else:
            np.testing.assert_allclose(v.numpy(), ref, atol=1e-4, rtol=1e-4, err_msg=k)
    loss, comp = cr.epipolar_loss(proc, F1, F2, (H, W))
    np.testing.assert_allclose(loss.numpy(), d[tag + "_epi_loss"], rtol=1e-4)
    for k, v in comp.items():
        np.testing.assert_allclose(v.numpy(), d["%s_epi_%s" % (tag, k)], rtol=1e-4, err_msg=k)


@pytest.mark.parametrize("tag", ["s", "f"])
def test_disk_loss_oracle(tag):
    d = np.load(os.path.join(GOLDEN, "correlation.npz"))
    b, H, W, xf1, xf2, kp1, kp2, F1, F2 = _inputs(tag)
    g = lambda k: torch.from_numpy(d["%s_%s" % (tag, k)])  # noqa: E731
    loss, comp = cr.disk_loss(kp1, kp2, xf1, xf2, F1, F2, g("prop1").long(), g("prop2").long(),
                              g("acc1"), g("acc2"))
    np.testing.assert_allclose(loss.numpy(), d[tag + "_disk_loss"], rtol=1e-4)
    for k in ("reinforce", "kp_penalty", "n_kps"):
        np.testing.assert_allclose(comp[k].numpy(), d["%s_disk_%s" % (tag, k)], rtol=1e-4)
