"""Keypoint-head training step (config 5, configs/train_kp.yaml).

CPU: the oracle (oracle/train_ref.py) against the reference's own autograd
gradients (tests/golden/train_kp.npz from tests/golden/gen_golden.py:
reference KeypointDet + DiskLoss, draws replayed) -- pins the oracle.
GPU: the HIP step (DiskLoss gradient, head backward kernels, SGD) against the
same fixture and against the oracle; determinism; the packing round trip.

Tolerances: gradients are compared per tensor as max|g - g_ref| <= 2e-3 *
max|g_ref| (fp32 sums over up to 4.9 M pixels in a different order; the
weight gradients are O(0.1-1)).  The conv biases feed an InstanceNorm, so
their exact gradient is 0 (conv3 too: norm3) and the reference's is fp32
noise (~1e-8): they
are compared with an absolute 1e-5 scaled by the layer's weight-gradient max.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

CASES = {"a": (2, 64, 96, 5, 300), "b": (1, 96, 128, 6, 301)}
KEYS = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "conv3.weight",
        "conv3.bias", "relu.weight", "convimg.weight", "convimg.bias"]


def _case(tag):
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.weights import seeded_image
    b, H, W, fseed, _ = CASES[tag]
    im1 = torch.from_numpy(np.stack([seeded_image(10 + i + 7 * fseed, H, W) for i in range(b)]))
    im2 = torch.from_numpy(np.stack([seeded_image(20 + i + 7 * fseed, H, W) for i in range(b)]))
    F1, F2 = synthetic_fundamental(b, H, W, fseed)
    d = np.load(os.path.join(GOLDEN, "train_kp.npz"))
    draws = [torch.from_numpy(d["%s_%s" % (tag, k)]) for k in ("prop1", "prop2", "acc1", "acc2")]
    return d, b, H, W, im1, im2, torch.from_numpy(F1), torch.from_numpy(F2), draws


def _assert_grads(got, d, tag, rel=2e-3):
    for k in KEYS:
        ref = d["%s_grad_%s" % (tag, k)]
        g = np.asarray(got[k]).reshape(ref.shape)
        if k.endswith(".bias"):
            wmax = np.abs(d["%s_grad_%s" % (tag, k.replace("bias", "weight"))]).max()
            assert np.abs(g - ref).max() <= 1e-5 * max(1.0, wmax), k
            continue
        scale = max(np.abs(ref).max(), 1e-6)
        err = np.abs(g - ref).max()
        assert err <= rel * scale, "%s: max err %.3e vs scale %.3e" % (k, err, scale)


@pytest.mark.parametrize("tag", list(CASES))
def test_oracle_train_step_vs_reference(tag):
    from oracle import train_ref
    from posfeat_amd.weights import seeded_state_dicts
    d, b, H, W, im1, im2, F1, F2, draws = _case(tag)
    bb, hd = seeded_state_dicts(0)
    p1, p2, a1, a2 = draws
    loss, grads, new, lps = train_ref.head_step(bb, hd, im1, im2, F1, F2,
                                                (p1.long(), p2.long(), a1, a2))
    np.testing.assert_allclose(lps[0].numpy(), d[tag + "_lp1"], atol=1e-5)
    np.testing.assert_allclose(float(loss), float(d[tag + "_loss"]), rtol=1e-4)
    # 5e-4: the oracle and the reference both run torch-CPU fp32, but conv
    # weight gradients over 2x96x128 pixels sum in BLAS/oneDNN order, which
    # differs between host CPUs (2.3e-4 relative on conv2.weight on an EPYC
    # host vs the Xeon the fixture was made on)
    _assert_grads({k: v.numpy() for k, v in grads.items()}, d, tag, rel=5e-4)


def test_pack_head_roundtrip():
    """unpack_head(pack_head(sd)) == sd: the packed gradient layout maps back
    onto the reference's localheader state-dict keys."""
    from posfeat_amd import weights
    specs = _fake_specs()
    _, hd = weights.seeded_state_dicts(3, as_torch=False)
    total = max(s[6] + max(s[1], 1) for s in specs) + 64
    region = weights.pack_head(hd, specs, total)
    back = weights.unpack_head(region, specs)
    for k in hd:
        np.testing.assert_array_equal(back[k].reshape(hd[k].shape), hd[k], err_msg=k)


def _fake_specs():
    """The head part of the engine's layer table, recomputed on the host (same
    rounding as engine.hip SpecTable) so the round trip runs without the GPU."""
    from posfeat_amd import _lib
    try:
        return _lib.model_specs()
    except Exception:  # pragma: no cover - library missing
        pytest.skip("libposfeat_hip.so not built")


# ------------------------------------------------------------------ GPU
def _gpu_step(gpu, tag, update=False, lr=1e-3):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.training import KeypointTrainStep
    from posfeat_amd.weights import seeded_state_dicts
    d, b, H, W, im1, im2, F1, F2, draws = _case(tag)
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device=gpu, train=True)
    step = KeypointTrainStep(eng, lr=lr)
    out, grad = step.step(im1.to(gpu), im2.to(gpu), F1, F2, epoch=1, draws=draws, update=update)
    torch.cuda.synchronize()
    return d, eng, out.cpu().numpy(), grad.cpu().numpy().copy()


@pytest.mark.gpu
@pytest.mark.parametrize("tag", list(CASES))
def test_gpu_train_step_grads_vs_reference(gpu, tag):
    from posfeat_amd import _lib, weights
    d, eng, out, grad = _gpu_step(gpu, tag)
    np.testing.assert_allclose(out[0], float(d[tag + "_loss"]), rtol=2e-4, atol=1e-4)
    np.testing.assert_allclose(out[1], float(d[tag + "_reinforce"]), rtol=2e-4, atol=1e-4)
    np.testing.assert_allclose(out[3], float(d[tag + "_n_kps"]), rtol=0, atol=0)
    got = weights.unpack_head(grad, _lib.model_specs())
    _assert_grads(got, d, tag)


@pytest.mark.gpu
def test_gpu_train_step_deterministic_and_sgd(gpu):
    from posfeat_amd import _lib, weights
    from posfeat_amd.weights import seeded_state_dicts
    _, eng, out1, g1 = _gpu_step(gpu, "a")
    _, eng2, out2, g2 = _gpu_step(gpu, "a", update=True, lr=0.5)
    np.testing.assert_array_equal(g1, g2)
    np.testing.assert_array_equal(out1, out2)
    # the update is w - lr * g on the head region only
    _, hd = seeded_state_dicts(0)
    new = weights.unpack_head(eng2.head_weights().cpu().numpy(), _lib.model_specs())
    for k in hd:
        np.testing.assert_allclose(new[k].reshape(hd[k].shape),
                                   hd[k].numpy() - 0.5 * weights.unpack_head(
                                       g2, _lib.model_specs())[k].reshape(hd[k].shape),
                                   rtol=1e-6, atol=1e-6, err_msg=k)


@pytest.mark.gpu
def test_gpu_wgrad_vs_torch(gpu):
    """posfeat_conv_wgrad (MFMA weight gradient, packed K order) against torch's
    conv2d weight gradient in fp64: the three head layer shapes and two 1x1
    shapes on the bf16x6 row tiles."""
    import ctypes
    from posfeat_amd import _lib, weights
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    rs = np.random.RandomState(0)
    # 3x3: the halo kernels (and Cin = 4: the fp32 row tiles); 1x1 with 128 x
    # 128 tiles: the bf16x6 row-tile kernel (conv_wgrad_bf6_kernel), incl. a
    # ragged last pixel chunk and several pixel splits
    for (n, h, w, cin, cout, k) in ((2, 20, 36, 256, 128, 3), (1, 17, 23, 192, 192, 3),
                                    (2, 24, 40, 4, 64, 3), (2, 20, 37, 256, 128, 1),
                                    (1, 60, 80, 512, 256, 1)):
        x = rs.randn(n, cin, h, w).astype(np.float32)
        if cin == 4:
            x[:, 3] = 0.0
        dy = rs.randn(n, cout, h, w).astype(np.float32)
        xt = torch.from_numpy(x).double().requires_grad_(True)
        wt = torch.zeros(cout, cin, k, k, dtype=torch.float64, requires_grad=True)
        y = torch.nn.functional.conv2d(xt, wt, padding=(k - 1) // 2)
        y.backward(torch.from_numpy(dy).double())
        ref_w = wt.grad.numpy()
        ref_b = dy.astype(np.float64).sum((0, 2, 3))
        xd = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 3, 1))).to(gpu)
        dyd = torch.from_numpy(np.ascontiguousarray(dy.transpose(0, 2, 3, 1))).to(gpu)
        kpad = lib().posfeat_conv_packed_k(cin, k, k)
        dw = torch.empty(cout * kpad, device=gpu)
        db = torch.empty(cout, device=gpu)
        need = lib().posfeat_conv_wgrad_workspace(n, h, w, cin, cout, k, k)
        ws = torch.empty(need, dtype=torch.uint8, device=gpu)
        check(lib().posfeat_conv_wgrad(ptr(dyd), cout, ptr(xd), cin, n, h, w, cin, cout, k, k,
                                       ptr(dw), ptr(db), ptr(ws), need, stream_ptr()))
        torch.cuda.synchronize()
        got = weights.unpack_conv(dw.cpu().numpy(), cout, cin, k, k)
        if cin == 4:
            ref_w = ref_w[:, :3]
            got = got[:, :3]
        scale = np.abs(x).max() * np.abs(dy).max() * n * h * w
        assert np.abs(got - ref_w).max() <= 2e-6 * scale
        assert np.abs(db.cpu().numpy() - ref_b).max() <= 2e-6 * np.abs(dy).max() * n * h * w


@pytest.mark.gpu
def test_gpu_wino_wgrad_vs_torch(gpu):
    """posfeat_conv3x3_wino_wgrad (F(4x4,3x3) weight gradient: dY transform,
    36 split transform-domain GEMMs, G^T dU G into the packed K order) against
    torch's fp64 conv2d weight/bias gradient; the last case splits the tile
    reduction (nsplit 3)."""
    from posfeat_amd import weights
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    rs = np.random.RandomState(1)
    for (n, h, w, cin, cout) in ((2, 16, 20, 128, 128), (1, 12, 24, 256, 128),
                                 (4, 64, 96, 128, 128)):
        x = rs.randn(n, cin, h, w).astype(np.float32)
        dy = rs.randn(n, cout, h, w).astype(np.float32)
        xt = torch.from_numpy(x).double()
        wt = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
        torch.nn.functional.conv2d(xt, wt, padding=1).backward(torch.from_numpy(dy).double())
        ref_w = wt.grad.numpy()
        ref_b = dy.astype(np.float64).sum((0, 2, 3))
        xd = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 3, 1))).to(gpu)
        dyd = torch.from_numpy(np.ascontiguousarray(dy.transpose(0, 2, 3, 1))).to(gpu)
        kpad = lib().posfeat_conv_packed_k(cin, 3, 3)
        dw = torch.full((cout * kpad,), float("nan"), device=gpu)
        db = torch.empty(cout, device=gpu)
        need = lib().posfeat_wino_wgrad_workspace(n, h, w, cin, cout)
        assert need > 0
        ws = torch.empty(need, dtype=torch.uint8, device=gpu)
        check(lib().posfeat_conv3x3_wino_wgrad(ptr(dyd), cout, ptr(xd), cin, n, h, w, cin, cout,
                                               ptr(dw), ptr(db), ptr(ws), need, stream_ptr()))
        torch.cuda.synchronize()
        got = weights.unpack_conv(dw.cpu().numpy(), cout, cin, 3, 3)
        # |dw| sums n*h*w products of unit normals: rms sqrt(n h w); the
        # Winograd transforms grow the fp32 rounding by ~10x over direct
        err = np.abs(got - ref_w).max() / np.sqrt(n * h * w)
        assert err <= 2e-4, err
        assert np.abs(db.cpu().numpy() - ref_b).max() <= 1e-4 * np.sqrt(n * h * w)

