"""Both training steps at the benchmarked size (bs = 8 pairs, 480x640): the
configuration bench.py's train_kp / train_desc lines time, which the gradient
fixtures (small sizes) do not reach.  Checked: finite loss and gradients,
bit-identical results for a repeated step from the same state and draws
(deterministic reductions, no atomics in the reductions that feed the
gradient), the gradient is not trivially zero, and the fused keypoint step
equals the autograd plug point (model.forward + DiskLoss + backward) on the
same draws.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, H, W = 8, 480, 640


def _pairs(gpu, seed):
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.weights import seeded_image
    im1 = torch.from_numpy(np.stack([seeded_image(seed + i, H, W) for i in range(B)])).to(gpu)
    im2 = torch.from_numpy(np.stack([seeded_image(seed + 50 + i, H, W) for i in range(B)])).to(gpu)
    F1, F2 = [torch.from_numpy(f).to(gpu) for f in synthetic_fundamental(B, H, W, seed)]
    return im1, im2, F1, F2


def test_kp_train_step_bs8_full_size(gpu):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.training import KeypointTrainStep
    from posfeat_amd.weights import seeded_state_dicts
    im1, im2, F1, F2 = _pairs(gpu, 500)
    n = (H // 8) * (W // 8)
    g = torch.Generator(device="cpu").manual_seed(7)
    draws = (torch.randint(0, 64, (B, n), generator=g), torch.randint(0, 64, (B, n), generator=g),
             (torch.rand(B, n, generator=g) < 0.5), (torch.rand(B, n, generator=g) < 0.5))
    bb, hd = seeded_state_dicts(0)
    res = []
    for _ in range(2):
        eng = ExtractionEngine(bb, hd, device=gpu, train=True)
        out, grad = KeypointTrainStep(eng, lr=1e-3).step(im1, im2, F1, F2, epoch=1, draws=draws,
                                                         update=False)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy().copy(), grad.cpu().numpy().copy()))
        eng.close()
    (o1, g1), (o2, g2) = res
    assert np.isfinite(o1).all() and np.isfinite(g1).all()
    assert np.abs(g1).max() > 0
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(g1, g2)
    # the autograd plug point on the same draws gives the same gradient
    from posfeat_amd import networks
    from posfeat_amd.losses import DiskLoss
    from posfeat_amd.training import DISK_DEFAULTS
    from test_gpu_trainer_plugpoints import MODEL_CONFIG
    m = networks.PoSFeat(MODEL_CONFIG, gpu)
    m.backbone.load_state_dict(bb)
    m.localheader.load_state_dict(hd)
    m.set_eval()
    m.localheader.train()
    inputs = {"im1": im1, "im2": im2, "F1": F1, "F2": F2}
    outputs = m.forward(inputs)
    outputs["epoch"] = 1
    loss, _ = DiskLoss(dict(DISK_DEFAULTS))(inputs, outputs, None, draws=draws)
    loss.backward()
    assert float(loss) == float(o1[0])
    from posfeat_amd import _lib, weights
    ref = weights.unpack_head(g1, _lib.model_specs())
    for k, p in m.localheader.named_parameters():
        np.testing.assert_array_equal(p.grad.cpu().numpy().reshape(-1), ref[k].reshape(-1),
                                      err_msg=k)


def test_desc_train_step_bs8_full_size(gpu):
    from posfeat_amd.training import (BackboneTrainer, DescriptorLossGrad, DESC_EPI_DEFAULTS,
                                      DESC_PRE_DEFAULTS)
    from posfeat_amd.weights import seeded_state_dicts
    im1, im2, F1, F2 = _pairs(gpu, 600)
    g = 16
    n = (H // g) * (W // g)
    gen = torch.Generator(device="cpu").manual_seed(8)
    draws = (torch.randint(0, g * g, (B, n), generator=gen).int(),
             torch.randint(0, g * g, (B, n), generator=gen).int(),
             torch.rand(B, n, 2, generator=gen), torch.rand(B, n, 2, generator=gen))
    bb, _ = seeded_state_dicts(0)
    loss = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
    res = []
    for _ in range(2):
        tr = BackboneTrainer(bb, B, H, W, device=gpu)
        out, _ = tr.step(im1, im2, F1, F2, loss, epoch=1, draws=draws, update=False)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy().copy(), tr.grad.cpu().numpy().copy(),
                    tr.stats.cpu().numpy().copy()))
        del tr
        torch.cuda.empty_cache()
    (o1, g1, s1), (o2, g2, s2) = res
    assert np.isfinite(o1).all() and np.isfinite(g1).all() and np.isfinite(s1).all()
    assert np.abs(g1).max() > 0 and 0 < o1[6] <= 1      # percent_w
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(g1, g2)
    np.testing.assert_array_equal(s1, s2)
