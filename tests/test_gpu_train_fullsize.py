"""Both training steps at the benchmarked size (bs = 8 pairs, 480x640): the
configuration bench.py's train_kp / train_desc lines time, which the gradient
fixtures (small sizes) do not reach.  Checked: finite loss and gradients,
bit-identical results for a repeated step from the same state and draws
(deterministic reductions, no atomics in the reductions that feed the
gradient), the gradient is not trivially zero, and the fused keypoint step
equals the autograd plug point (model.forward + DiskLoss + backward) on the
same draws; and the descriptor step's gradients against the same step in
fp64, per tensor within 3x the fp32 reference's own error (r12p against fp32:
worst tensor 3.6e-2 of its max, relative L2 2.3e-3 over all).
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


def test_desc_train_step_bs8_vs_torch_fp32(gpu):
    """The benchmarked descriptor step (bs 8 pairs, 480x640) against a plain
    PyTorch fp32 reference of the same step on the GPU: the oracle's
    train-mode ResUNet (oracle/model_ref.py, torch ops) and desc loss
    (oracle/desc_train_ref.py) under torch autograd, sharing the HIP step's
    window centres and loss weights (arg-max near-ties, as the fixture test
    does).  The loss within 2e-3 of the fp32 reference; every backbone
    gradient tensor within max(3 x the fp32 reference's own error, 1e-2) of
    the same backward run in fp64 (the bound of test_bb_train's fp64 fixture,
    this 13-block train-mode network's fp32 gradients carrying up to ~3e-2
    relative rounding noise of their own).  A tensor's noise is the larger
    error of two fp32 realisations of the reference (MIOpen's convolutions and
    PyTorch's native im2col + GEMM ones), at least the median over the tensors
    (each realisation is one sample of the rounding error).  All tensors
    together within 5e-3 relative L2 of fp64."""
    from oracle.desc_train_ref import desc_loss_grad, loss_weights
    from oracle.model_ref import resunet_forward
    from posfeat_amd.training import (BackboneTrainer, DescriptorLossGrad, DESC_EPI_DEFAULTS,
                                      DESC_PRE_DEFAULTS)
    from posfeat_amd.weights import seeded_state_dicts
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    im1, im2, F1, F2 = _pairs(gpu, 700)
    g = 16
    n = (H // g) * (W // g)
    gen = torch.Generator(device="cpu").manual_seed(9)
    draws = (torch.randint(0, g * g, (B, n), generator=gen).int(),
             torch.randint(0, g * g, (B, n), generator=gen).int(),
             torch.rand(B, n, 2, generator=gen), torch.rand(B, n, 2, generator=gen))
    bb, _ = seeded_state_dicts(0)
    tr = BackboneTrainer(bb, B, H, W, device=gpu)
    out, res = tr.step(im1, im2, F1, F2, DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS),
                       epoch=1, draws=draws, update=False)
    torch.cuda.synchronize()
    got = tr.grad_dict()
    del tr
    sd = {k: v.clone().to(gpu) for k, v in bb.items()}
    keys = [k for k, v in sd.items() if v.is_floating_point() and "running" not in k
            and "num_batches" not in k and not k.endswith("conv.bias") and k in got]
    params = {k: sd[k].requires_grad_(True) for k in keys}
    x1 = resunet_forward(sd, im1, train=True)["local_map"]
    x2 = resunet_forward(sd, im2, train=True)["local_map"]
    # the loss and its map gradient in fp32 on the host (the oracle's
    # correlation code is host torch), the network's backward on the GPU
    res = {k: v.cpu() for k, v in res.items()}
    F1c, F2c = F1.cpu(), F2.cpu()
    short = min(H, W)
    wts = [loss_weights(res["coord%d" % i], res["w%d" % i], res["w%d_std" % i],
                        res["valid%d" % i].bool(), Fm, short) for i, Fm in ((1, F1c), (2, F2c))]
    dd = (draws[0].long().view(B, H // g, W // g), draws[1].long().view(B, H // g, W // g),
          draws[2], draws[3])
    loss, g1, g2, _ = desc_loss_grad(x1.detach().cpu(), x2.detach().cpu(), F1c, F2c, (H, W),
                                     (H, W), *dd, centers=(res["l1_exp_n"], res["l2_exp_n"]),
                                     weights=wts)
    np.testing.assert_allclose(float(out[0]), float(loss), rtol=2e-3)
    grads = torch.autograd.grad([x1, x2], [params[k] for k in keys],
                                grad_outputs=[g1.to(gpu), g2.to(gpu)], allow_unused=True)
    g32 = {k: (None if gr is None else gr.detach().double().cpu().numpy())
           for k, gr in zip(keys, grads)}
    del grads, x1, x2, params
    # a second fp32 realisation of the reference backward: PyTorch's native
    # im2col + GEMM convolutions instead of MIOpen's (another summation order)
    sdb = {k: v.clone().to(gpu) for k, v in bb.items()}
    pb = {k: sdb[k].requires_grad_(True) for k in keys}
    with torch.backends.cudnn.flags(enabled=False):
        z1 = resunet_forward(sdb, im1, train=True)["local_map"]
        z2 = resunet_forward(sdb, im2, train=True)["local_map"]
        grads_b = torch.autograd.grad([z1, z2], [pb[k] for k in keys],
                                      grad_outputs=[g1.to(gpu), g2.to(gpu)], allow_unused=True)
    g32b = {k: (None if gr is None else gr.detach().double().cpu().numpy())
            for k, gr in zip(keys, grads_b)}
    del grads_b, z1, z2, pb
    torch.cuda.empty_cache()
    # the same network backward in fp64 (torch's native double convs on the
    # GPU), fed the same map gradients: the reference's own fp32 noise per
    # tensor is |g32 - g64|, and the HIP step must sit within 3x that noise
    # (floor 1e-2) of fp64 -- test_bb_train's fixture bound at this size
    sd64 = {k: v.clone().to(gpu).double() for k, v in bb.items()}
    p64 = {k: sd64[k].requires_grad_(True) for k in keys}
    y1 = resunet_forward(sd64, im1.double(), train=True)["local_map"]
    y2 = resunet_forward(sd64, im2.double(), train=True)["local_map"]
    grads64 = torch.autograd.grad([y1, y2], [p64[k] for k in keys],
                                  grad_outputs=[g1.to(gpu).double(), g2.to(gpu).double()],
                                  allow_unused=True)
    num = den = 0.0
    rows = []
    for k, gr in zip(keys, grads64):
        if gr is None:   # not on local_map's path (conv_coarse): no gradient either way
            assert g32[k] is None and not np.any(np.asarray(got[k])), k
            continue
        ref = gr.detach().cpu().numpy()
        gk = np.asarray(got[k], np.float64).reshape(ref.shape)
        mx = max(np.abs(ref).max(), 1e-30)
        noise = max(np.abs(g32[k] - ref).max(), np.abs(g32b[k] - ref).max()) / mx
        rows.append((float(np.abs(gk - ref).max() / mx), float(noise), k))
        num += float(((gk - ref) ** 2).sum())
        den += float((ref ** 2).sum())
    # a tensor's noise: the larger error of the two fp32 realisations (MIOpen,
    # native); each is one sample of the fp32 rounding error and can come out
    # small by chance, so it counts as at least the median over the tensors
    med = float(np.median([n for _, n, _ in rows]))
    bad, errs = [], []
    for e, noise, k in rows:
        tol_k = max(3.0 * max(noise, med), 1e-2)
        errs.append((e, noise, k))
        if e > tol_k:
            bad.append((k, round(e, 5), round(tol_k, 5)))
    print("largest relative errors vs fp64 (err, torch fp32 noise):",
          [(k, "%.2e" % e, "%.2e" % n) for e, n, k in sorted(errs)[-8:]],
          "median noise %.2e, largest err / max(noise, median): %.2f" % (
              med, max(e / max(n, med) for e, n, _ in rows)),
          "rel L2 %.2e" % np.sqrt(num / den))
    assert not bad, "tensors over max(3 x fp32 noise, 1e-2) (key, err, tol): %s" % bad
    assert np.sqrt(num / den) <= 5e-3, np.sqrt(num / den)
