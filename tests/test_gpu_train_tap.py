"""Keypoint-head backward on the extraction path's factorisation (traintap,
the default): head.conv2's upsampled part through the low-res tap GEMM and
its backward as the combine's adjoint + two low-res GEMMs, the image branch
through the 32-channel tap image (posfeat_amd/csrc/headgrad.hip).

Checked with a FIXED smooth upstream gradient dL/d local_point, so
the comparison isolates the head backward: against the reference KeypointDet
(networks/DeteNet.py:102-121, restated in oracle/model_ref.py) under torch
autograd in fp64 on the engine's own backbone maps, and against the materialised-input path
(POSFEAT_TRAINTAP=0: direct 3x3 weight / input gradients over
cat[up4(L), G]).  Shapes with many interior tiles, ragged low-res column
blocks (w/4 % 8 != 0) and several images (per-image IN statistics and image
moments must not mix).

(Through DiskLoss the two GPU paths differ by up to ~3e-3 of a gradient's
scale at 2 pairs of 128 x 160: DiskLoss multiplies descriptor cosines by 60
and the local_point maps of the two forwards differ in the last bits; both
then sit ~1e-2 from the CPU oracle, whose backbone maps differ more.  The
end-to-end step is pinned at the fixture sizes by tests/test_train_kp.py.)
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "conv3.weight",
        "conv3.bias", "relu.weight", "convimg.weight", "convimg.bias"]


def _imgs(b, H, W, seed):
    from posfeat_amd.weights import seeded_image
    return torch.from_numpy(np.stack([seeded_image(seed + i, H, W) for i in range(b)]))


def _dlp(b, H, W, seed):
    """a smooth upstream gradient: the head gradient is then a coherent sum
    (a white-noise dL/d local_point makes it a random walk whose value is
    small against its terms, and every PReLU kink that fp32 and fp64 place
    differently moves it by O(1) of a term)"""
    y = torch.arange(H, dtype=torch.float64)[:, None] / H
    x = torch.arange(W, dtype=torch.float64)[None, :] / W
    out = [1.0 + 0.5 * torch.sin(2 * np.pi * (x + 0.13 * i + 0.01 * seed)) *
           torch.cos(2 * np.pi * y) for i in range(b)]
    return torch.stack(out)[:, None].float()


def _gpu_grads(gpu, monkeypatch, flag, imgs, dlp):
    from posfeat_amd import _lib, weights
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_state_dicts
    monkeypatch.setenv("POSFEAT_TRAINTAP", flag)
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device=gpu, train=True)
    res = eng.run(imgs.to(gpu).float(), outputs=("local_map", "local_map_small"))
    lp = res["local_point"].cpu().numpy().copy()
    x = torch.cat([res["local_map"], res["local_map_small"]], 1).cpu()
    grad = eng.head_backward(dlp.to(gpu))
    torch.cuda.synchronize()
    got = weights.unpack_head(grad.cpu().numpy().copy(), _lib.model_specs())
    eng.close()
    return lp, got, x


def _oracle_grads(imgs, dlp, x, dtype=torch.float64):
    """the reference KeypointDet (fp64, or fp32 for the noise floor) on the
    ENGINE's backbone maps x"""
    from oracle.model_ref import keypointdet_forward
    from posfeat_amd.weights import seeded_state_dicts
    _, hd = seeded_state_dicts(0)
    x = x.to(dtype)
    params = {k: v.clone().to(dtype).requires_grad_(True) for k, v in hd.items()}
    lp = keypointdet_forward(params, x, imgs.to(dtype))
    grads = torch.autograd.grad(lp, [params[k] for k in hd], dlp.to(dtype))
    return {k: g.double().numpy() for k, g in zip(hd, grads)}


def _compare(got, ref, what, rel, floor=None):
    """per tensor max|got - ref| <= rel * max|ref|, or <= 3x the reference's
    own fp32 error (floor[k], absolute) where that is larger"""
    bad = []
    for k in KEYS:
        g, r = np.asarray(got[k]).reshape(-1), np.asarray(ref[k]).reshape(-1)
        assert np.isfinite(g).all(), k
        if k.endswith(".bias"):  # conv biases into an InstanceNorm: exact gradient 0
            wmax = np.abs(np.asarray(ref[k.replace("bias", "weight")])).max()
            err, lim = np.abs(g - r).max(), 1e-5 * max(1.0, wmax)
        else:
            err, lim = np.abs(g - r).max(), rel * max(np.abs(r).max(), 1e-6)
            if floor is not None:
                lim = max(lim, 3.0 * floor[k])
        print("%s %-16s err %.3e  limit %.3e" % (what, k, err, lim))
        if err > lim:
            bad.append(k)
    return bad


@pytest.mark.parametrize("shape", [(4, 128, 160), (2, 96, 208)])
def test_traintap_backward(gpu, monkeypatch, shape):
    b, H, W = shape
    imgs, dlp = _imgs(b, H, W, 700 + H), _dlp(b, H, W, 7 + W)
    lp_old, g_old, x = _gpu_grads(gpu, monkeypatch, "0", imgs, dlp)
    lp_tap, g_tap, _ = _gpu_grads(gpu, monkeypatch, "1", imgs, dlp)
    np.testing.assert_allclose(lp_tap, lp_old, rtol=1e-4, atol=1e-5)
    g_or = _oracle_grads(imgs, dlp, x)
    # the same reference in fp32 (torch CPU): its own error vs fp64 is the
    # noise floor of this input (r4c, 2 x 96 x 208: 0.70 on conv1.weight of
    # scale 176 -- a badly conditioned IN channel -- which the GPU matches)
    # One fp32 run samples that error once; it swings by 30x with the rounding
    # of the same maps (r5g: 0.025 where r4c saw 0.70, after an upstream
    # change moved the backbone maps by 1e-6), so the floor is the largest of
    # the fp32 reference's errors over x and three copies of x perturbed by
    # one fp32 ulp (relative 2^-23, seeded): the spread of fp32 outcomes
    g_32 = _oracle_grads(imgs, dlp, x, torch.float32)
    _compare(g_32, g_or, "cpu32-vs-ref64", 2e-3)
    floor = {k: float(np.abs(np.asarray(g_32[k]) - np.asarray(g_or[k])).max()) for k in KEYS}
    gen = torch.Generator().manual_seed(H * W)
    for _ in range(3):
        u = (torch.rand(x.shape, generator=gen, dtype=torch.float64) * 2 - 1) * 2.0 ** -23
        g_p = _oracle_grads(imgs, dlp, (x.double() * (1 + u)).float(), torch.float32)
        for k in KEYS:
            floor[k] = max(floor[k], float(np.abs(np.asarray(g_p[k]) - np.asarray(g_or[k])).max()))
    print("fp32 floors: " + " ".join("%s %.3e" % (k, floor[k]) for k in KEYS))
    # The weight gradients contract zero-mean IN-backward fields against
    # inputs with large means (heavy cancellation): in fp32 BOTH GPU paths sit
    # up to ~8e-4 of a tensor's scale from the fp64 reference (measured r3h:
    # conv2 / convimg weights at 2 x 96 x 208, the two paths within 5 % of
    # each other's error), so the bound is the golden test's 2e-3 -- or 3x the
    # fp32 reference's own error on this input where that is larger; the two
    # GPU paths differ by summation order only (<= 4e-4 measured)
    #
    # 2 x 96 x 208 is the ill-conditioned case: both GPU paths sit 0.63 of
    # scale 176 (3.6e-3) from fp64 on conv1.weight (r5g, and ~0.7 in r4c),
    # where torch-CPU fp32 was itself 0.70 off in r4c and 0.025 in r5g on
    # maps 1e-6 apart (the perturbed-copy floor above does not reach such
    # excursions: they come from the IN statistics of conv1's output, not
    # from x).  Bound there: 5e-3 of scale (the r4c fp32 excursion, 4.0e-3,
    # plus margin); 2e-3 on the well-conditioned shape
    rel = 2e-3 if (H, W) == (128, 160) else 5e-3
    bad = _compare(g_tap, g_old, "tap-vs-old", 1e-3)
    bad += _compare(g_tap, g_or, "tap-vs-ref64", rel, floor)
    bad += ["old:" + k for k in _compare(g_old, g_or, "old-vs-ref64", rel, floor)]
    assert not bad, bad


def test_traintap_deterministic(gpu, monkeypatch):
    imgs, dlp = _imgs(4, 64, 96, 333), _dlp(4, 64, 96, 5)
    _, g1, _ = _gpu_grads(gpu, monkeypatch, "1", imgs, dlp)
    _, g2, _ = _gpu_grads(gpu, monkeypatch, "1", imgs, dlp)
    for k in KEYS:
        np.testing.assert_array_equal(g1[k], g2[k], err_msg=k)
