"""GPU parity of the individual HIP kernels, through the C ABI.

Floating-point kernels (conv, sampler, layout) are compared with a plain
torch fp32/fp64 CPU reference of the same op; the detector (integer/index
work) must be bit-exact against the numpy oracle and the golden fixtures
generated from the reference's own generate_kpts_single.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _conv_ref64(x, w, b, stride, pad, res=None, act="none"):
    y = F.conv2d(x.double(), w.double(), b.double() if b is not None else None, stride=stride,
                 padding=pad)
    if res is not None:
        y = y + res.double()
    if act == "relu":
        y = torch.relu(y)
    elif act == "elu":
        y = F.elu(y)
    bound = F.conv2d(x.double().abs(), w.double().abs(), None, stride=stride, padding=pad)
    return y, bound


CONV_CASES = [
    # n, h, w, cin, cout, k, stride, act, residual, in_extra, out_extra
    (2, 17, 23, 64, 96, 3, 1, "none", False, 0, 0),
    (1, 20, 30, 256, 64, 1, 1, "relu", True, 0, 0),
    (2, 19, 21, 128, 128, 3, 2, "relu", False, 64, 0),
    (1, 33, 47, 3, 64, 7, 2, "relu", False, 1, 0),      # stem: cin 3 padded to 4
    (1, 24, 40, 3, 64, 3, 1, "none", False, 1, 192),    # convimg into a 256-wide slice
    (1, 16, 20, 512, 256, 1, 2, "none", False, 0, 0),   # downsample 1x1 s2
    (1, 12, 16, 1024, 512, 3, 1, "elu", False, 0, 0),
    (1, 256, 256, 64, 128, 3, 1, "elu", True, 0, 0),    # 128x128-tile path
    (1, 30, 40, 192, 192, 3, 1, "none", False, 0, 0),   # cout 192 (tile guard)
    (3, 21, 37, 96, 128, 3, 1, "relu", True, 8, 64),    # halo: slice in/out, ragged patches
    (2, 9, 17, 32, 64, 3, 1, "elu", False, 0, 0),       # halo: 8x16 patches, both edges partial
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_vs_torch(gpu, case):
    from posfeat_amd import ops
    n, h, w, cin, cout, k, s, act, has_res, in_extra, out_extra = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = (k - 1) // 2
    oh, ow = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
    res = torch.randn(n, cout, oh, ow, generator=g) if has_res else None
    ref, bound = _conv_ref64(x, wt, b, s, pad, res, act)
    cinp = (cin + 3) // 4 * 4
    xcs = cinp + in_extra * 4
    xd = torch.zeros(n, h, w, xcs)
    xd[..., :cin] = x.permute(0, 2, 3, 1)
    xd = xd.to(gpu)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    out = torch.full((n, oh, ow, cout + out_extra), 7.0, device=gpu)
    rd = res.permute(0, 2, 3, 1).contiguous().to(gpu) if has_res else None
    ops.conv2d_nhwc(xd, wp, bp, cout, k, k, stride=s, pad=pad, act=act, res=rd, out=out, cin=cinp)
    torch.cuda.synchronize()
    got = out[..., :cout].permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 2e-6 * bound + 1e-6
    assert torch.all(err <= tol), "max err %g (bound %g)" % (err.max(), (err / tol).max())
    if out_extra:
        assert torch.all(out[..., cout:] == 7.0).item(), "wrote outside its channel slice"


DUAL_CASES = [
    # n, oh, ow, k1 (conv3 input), k2 (downsample input), cout, stride of the downsample
    (2, 24, 40, 64, 64, 256, 1),      # layer1.0 (ragged last tile: 1920 rows)
    (1, 15, 20, 128, 256, 512, 2),    # layer2.0
    (2, 8, 10, 256, 512, 1024, 2),    # layer3.0
]


@pytest.mark.parametrize("case", DUAL_CASES)
def test_conv1x1_dual_vs_torch(gpu, case):
    """A bottleneck's conv3 + downsample as one two-source GEMM
    (posfeat_conv1x1_dual) vs relu(conv3(t) + conv_ds(x) + biases) in fp64,
    the bound of test_conv_vs_torch over both K ranges."""
    from posfeat_amd import ops
    n, oh, ow, k1, k2, cout, s = case
    h2, w2 = (oh - 1) * s + 1 + (s - 1), (ow - 1) * s + 1 + (s - 1)
    g = torch.Generator().manual_seed(hash(case) % 1000)
    t = torch.randn(n, k1, oh, ow, generator=g)
    x = torch.randn(n, k2, h2, w2, generator=g)
    w1 = torch.randn(cout, k1, 1, 1, generator=g) * (2.0 / k1) ** 0.5
    w2 = torch.randn(cout, k2, 1, 1, generator=g) * (2.0 / k2) ** 0.5
    b1 = torch.randn(cout, generator=g) * 0.1
    b2 = torch.randn(cout, generator=g) * 0.1
    r1, bd1 = _conv_ref64(t, w1, b1, 1, 0)
    r2, bd2 = _conv_ref64(x, w2, b2, s, 0)
    ref = torch.relu(r1 + r2)
    bound = bd1 + bd2
    out = ops.conv1x1_dual(t.permute(0, 2, 3, 1).contiguous().to(gpu),
                           x.permute(0, 2, 3, 1).contiguous().to(gpu), w1[:, :, 0, 0].to(gpu),
                           w2[:, :, 0, 0].to(gpu), b1.to(gpu), b2.to(gpu), stride2=s, act="relu")
    torch.cuda.synchronize()
    got = out.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 2e-6 * bound + 1e-6
    assert torch.all(err <= tol), "max err %g (bound %g)" % (err.max(), (err / tol).max())


WINO_CASES = [
    # n, h, w, cin, cout, act, in_extra, out_extra
    (2, 16, 24, 64, 64, "none", 0, 0),       # F(4x4)
    (2, 18, 22, 64, 64, "elu", 0, 0),        # F(2x2) (not multiples of 4)
    (1, 30, 40, 1024, 512, "elu", 0, 512),   # upconv3 shape into a concat slice
    (2, 14, 10, 512, 256, "elu", 64, 0),     # ragged tile grid, strided input
    (1, 60, 80, 512, 256, "relu", 0, 256),
]


@pytest.mark.parametrize("case", WINO_CASES)
def test_conv3x3_wino_vs_torch(gpu, case):
    """Winograd path (wino.hip: F(4x4,3x3) when h, w % 4 == 0, else F(2x2,3x3))
    against the fp64 conv.  Transform-domain sums grow the fp32 rounding
    (F(4x4)'s coefficients reach 8 and 1/24), so the bound is a multiple of the
    direct conv's."""
    from posfeat_amd import ops
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    n, h, w, cin, cout, act, in_extra, out_extra = case
    g = torch.Generator().manual_seed(sum(case[:5]))
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref, bound = _conv_ref64(x, wt, b, 1, 1, None, act)
    xcs = cin + in_extra
    xd = torch.zeros(n, h, w, xcs)
    xd[..., :cin] = x.permute(0, 2, 3, 1)
    xd = xd.to(gpu)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    U = torch.empty(36 * cout * cin, device=gpu)
    check(lib().posfeat_wino_weights(ptr(wp), cout, cin, h, w, ptr(U), stream_ptr()))
    need = lib().posfeat_wino_workspace(n, h, w, cin, cout)
    ws = torch.empty(need, dtype=torch.uint8, device=gpu)
    out = torch.full((n, h, w, cout + out_extra), 7.0, device=gpu)
    actc = {"none": 0, "relu": 1, "elu": 2}[act]
    check(lib().posfeat_conv3x3_wino(ptr(xd), xcs, n, h, w, cin, ptr(U), ptr(bp), cout, actc,
                                     ptr(out), cout + out_extra, ptr(ws), need, stream_ptr()))
    torch.cuda.synchronize()
    got = out[..., :cout].permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 3e-5 * bound + 1e-6
    assert torch.all(err <= tol), "max err %g (ratio %g)" % (err.max(), (err / tol).max())
    if out_extra:
        assert torch.all(out[..., cout:] == 7.0).item(), "wrote outside its channel slice"


WINO6_CASES = [
    # n, h, w, cin, cout, act, in_extra, out_extra
    (2, 18, 24, 64, 64, "none", 0, 0),       # whole 6x6 tiles
    (2, 20, 26, 64, 128, "elu", 0, 0),       # last tile row / column cut
    (1, 13, 7, 96, 64, "relu", 32, 0),       # odd sizes, strided input
    (1, 30, 40, 1024, 512, "elu", 0, 512),   # upconv3 shape into a concat slice
    (2, 60, 80, 512, 256, "elu", 0, 256),    # upconv2 / iconv2 shape (80 = 13 tiles + 2)
    (1, 24, 32, 192, 192, "none", 0, 0),     # head.conv1
]


@pytest.mark.parametrize("case", WINO6_CASES)
def test_conv3x3_wino6_vs_torch(gpu, case):
    """Winograd F(6x6,3x3) (wino.hip, the extraction engine's decoder and
    head.conv1) against the fp64 conv, with the F(4x4) test's bound: B^T and
    A^T are exact in fp32 (quarters, powers of two to 32), G carries ninths and
    1/90; measured errors sit well inside it."""
    from posfeat_amd import ops
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    n, h, w, cin, cout, act, in_extra, out_extra = case
    g = torch.Generator().manual_seed(sum(case[:5]) + 6)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref, bound = _conv_ref64(x, wt, b, 1, 1, None, act)
    xcs = cin + in_extra
    xd = torch.zeros(n, h, w, xcs)
    xd[..., :cin] = x.permute(0, 2, 3, 1)
    xd = xd.to(gpu)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    U = torch.empty(64 * cout * cin, device=gpu)
    check(lib().posfeat_wino6_weights(ptr(wp), cout, cin, ptr(U), stream_ptr()))
    need = lib().posfeat_wino6_workspace(n, h, w, cin, cout)
    ws = torch.empty(need, dtype=torch.uint8, device=gpu)
    out = torch.full((n, h, w, cout + out_extra), 7.0, device=gpu)
    actc = {"none": 0, "relu": 1, "elu": 2}[act]
    check(lib().posfeat_conv3x3_wino6(ptr(xd), xcs, n, h, w, cin, ptr(U), ptr(bp), cout, actc,
                                      ptr(out), cout + out_extra, ptr(ws), need, stream_ptr()))
    torch.cuda.synchronize()
    got = out[..., :cout].permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 3e-5 * bound + 1e-6
    assert torch.all(err <= tol), "max err %g (ratio %g)" % (err.max(), (err / tol).max())
    print("wino6 %s: max err / bound %.2e" % (case, (err / bound.clamp_min(1e-30)).max()))
    if out_extra:
        assert torch.all(out[..., cout:] == 7.0).item(), "wrote outside its channel slice"


WINO6_EX_CASES = [
    # n, h, w, cin, cout, act, planes, up2
    (2, 18, 24, 64, 64, "none", 1, 0),       # three-plane U, whole tiles
    (1, 30, 40, 1024, 512, "elu", 1, 0),     # iconv3 shape, planes (the engine's default)
    (2, 60, 80, 512, 256, "elu", 1, 1),      # upconv2 shape: x2 upsample in the transform
    (1, 30, 40, 1024, 512, "elu", 1, 1),     # upconv3 shape
    (2, 20, 26, 64, 128, "relu", 0, 1),      # fp32 U + upsample, cut tiles
]


@pytest.mark.parametrize("case", WINO6_EX_CASES)
def test_conv3x3_wino6_planes_up2_vs_torch(gpu, case):
    """The extraction engine's F(6x6) variants: U as three bf16
    planes (planes = 1, the GEMM splitting V on the fly: bf16x6) and the
    decoder's x2 bilinear upsample (align_corners = True,
    DescNet.py:182-190) formed inside the input transform (up2 = 1), against
    the fp64 conv of the fp64-upsampled input, with test_conv3x3_wino6's
    bound."""
    from posfeat_amd import ops
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    n, h, w, cin, cout, act, planes, up2 = case
    g = torch.Generator().manual_seed(sum(case[:5]) + 60)
    hi, wi = (h // 2, w // 2) if up2 else (h, w)
    x = torch.randn(n, cin, hi, wi, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    xu = F.interpolate(x.double(), scale_factor=2, mode="bilinear",
                       align_corners=True) if up2 else x.double()
    assert xu.shape[-2:] == (h, w)
    ref, bound = _conv_ref64(xu, wt, b, 1, 1, None, act)
    xd = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    U = torch.empty(lib().posfeat_wino6_weights_floats(cin, cout, planes), device=gpu)
    check(lib().posfeat_wino6_weights_planes(ptr(wp), cout, cin, planes, ptr(U), stream_ptr()))
    need = lib().posfeat_wino6_workspace(n, h, w, cin, cout)
    ws = torch.empty(need, dtype=torch.uint8, device=gpu)
    out = torch.full((n, h, w, cout), 7.0, device=gpu)
    actc = {"none": 0, "relu": 1, "elu": 2}[act]
    check(lib().posfeat_conv3x3_wino6_ex(ptr(xd), cin, n, h, w, cin, ptr(U), planes, up2, ptr(bp),
                                         cout, actc, ptr(out), cout, ptr(ws), need, stream_ptr()))
    torch.cuda.synchronize()
    got = out.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 3e-5 * bound + 1e-6
    print("wino6 ex %s: max err / bound %.2e" % (case, (err / bound.clamp_min(1e-30)).max()))
    assert torch.all(err <= tol), "max err %g (ratio %g)" % (err.max(), (err / tol).max())
    # the plain fp32-U / materialised-upsample form of the same conv agrees
    if planes or up2:
        xm = xu.float().permute(0, 2, 3, 1).contiguous().to(gpu)
        U0 = torch.empty(64 * cout * cin, device=gpu)
        check(lib().posfeat_wino6_weights(ptr(wp), cout, cin, ptr(U0), stream_ptr()))
        out0 = torch.empty_like(out)
        check(lib().posfeat_conv3x3_wino6(ptr(xm), cin, n, h, w, cin, ptr(U0), ptr(bp), cout, actc,
                                          ptr(out0), cout, ptr(ws), need, stream_ptr()))
        torch.cuda.synchronize()
        d = (out0 - out).abs().max().item()
        assert d <= 2e-5 * float(bound.max()), d


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 18, 24, 128, 128), (1, 20, 26, 256, 128),
                                             (2, 60, 80, 512, 256)])
def test_conv3x3_wino6_wgrad_vs_torch_and_f4(gpu, n, h, w, cin, cout):
    """posfeat_conv3x3_wino6_wgrad (the training step's F(6x6) weight
    gradient: dY transform, 64 split transform-domain GEMMs, G^T dU G) against
    torch's fp64 conv2d weight/bias gradient, with the F(4x4) test's bound
    (tests/test_train_kp.py), and against the F(4x4) weight gradient where
    h, w % 4 == 0."""
    from posfeat_amd import weights
    from posfeat_amd._lib import check, lib, ptr, stream_ptr
    rs = np.random.RandomState(n * h + w + cin)
    x = rs.randn(n, cin, h, w).astype(np.float32)
    dy = rs.randn(n, cout, h, w).astype(np.float32)
    xt = torch.from_numpy(x).double()
    wt = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xt, wt, padding=1).backward(torch.from_numpy(dy).double())
    ref_w = wt.grad.numpy()
    ref_b = dy.astype(np.float64).sum((0, 2, 3))
    xd = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 3, 1))).to(gpu)
    dyd = torch.from_numpy(np.ascontiguousarray(dy.transpose(0, 2, 3, 1))).to(gpu)
    kpad = lib().posfeat_conv_packed_k(cin, 3, 3)

    def run(fn, wsfn):
        dw = torch.full((cout * kpad,), float("nan"), device=gpu)
        db = torch.empty(cout, device=gpu)
        need = wsfn(n, h, w, cin, cout)
        assert need > 0
        ws = torch.empty(need, dtype=torch.uint8, device=gpu)
        check(fn(ptr(dyd), cout, ptr(xd), cin, n, h, w, cin, cout, ptr(dw), ptr(db), ptr(ws), need,
                 stream_ptr()))
        torch.cuda.synchronize()
        return weights.unpack_conv(dw.cpu().numpy(), cout, cin, 3, 3), db.cpu().numpy()
    got, gb = run(lib().posfeat_conv3x3_wino6_wgrad, lib().posfeat_wino6_wgrad_workspace)
    err = np.abs(got - ref_w).max() / np.sqrt(n * h * w)
    print("wino6 wgrad %s: err %.2e" % ((n, h, w, cin, cout), err))
    assert err <= 2e-4, err
    assert np.abs(gb - ref_b).max() <= 1e-4 * np.sqrt(n * h * w)
    if h % 4 == 0 and w % 4 == 0:
        g4, _ = run(lib().posfeat_conv3x3_wino_wgrad, lib().posfeat_wino_wgrad_workspace)
        e4 = np.abs(g4 - ref_w).max() / np.sqrt(n * h * w)
        assert np.abs(got - g4).max() / np.sqrt(n * h * w) <= 2e-4 + e4


@pytest.mark.parametrize("act,has_res", [("elu", False), ("relu", True)])
def test_conv_splitk_vs_torch(gpu, act, has_res):
    """Deep-K shape that takes the split-K path (partials + ordered reduce)."""
    import ctypes
    from posfeat_amd import ops, _lib
    n, h, w, cin, cout = 1, 20, 24, 1024, 512
    d = _lib.ConvDesc(n=n, h=h, w=w, cin=cin, x_cstride=cin, cout=cout, kh=3, kw=3, stride=1,
                      pad=1, y_cstride=cout, res_cstride=cout if has_res else 0, act=0)
    assert _lib.lib().posfeat_conv2d_workspace(ctypes.byref(d)) > 0, "shape should split"
    g = torch.Generator().manual_seed(21)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, cout, h, w, generator=g) if has_res else None
    ref, bound = _conv_ref64(x, wt, b, 1, 1, res, act)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    rd = res.permute(0, 2, 3, 1).contiguous().to(gpu) if has_res else None
    xd = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    out = ops.conv2d_nhwc(xd, wp, bp, cout, 3, 3, act=act, res=rd, allow_split=True)
    got = out.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    assert torch.all(err <= 2e-6 * bound + 1e-6), "max err %g" % err.max()
    again = ops.conv2d_nhwc(xd, wp, bp, cout, 3, 3, act=act, res=rd, allow_split=True)
    assert torch.equal(out, again)


@pytest.mark.parametrize("n,h,w,cin,cout", [(3, 20, 28, 64, 128),     # tiles cross images
                                             (2, 48, 64, 192, 192),
                                             (1, 96, 80, 4, 64)])
def test_conv_fused_instnorm_stats(gpu, n, h, w, cin, cout):
    """Conv epilogue IN statistics == torch instance_norm statistics."""
    from posfeat_amd import ops
    g = torch.Generator().manual_seed(n * 7 + h)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) + 0.5
    ref = F.conv2d(x.double(), wt.double(), b.double(), padding=1)
    mu = ref.mean((2, 3))
    var = ref.var((2, 3), unbiased=False)
    xd = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    y, mean, rstd = ops.conv2d_nhwc_instnorm_stats(xd, wp, bp, cout, 3, 3)
    torch.cuda.synchronize()
    assert torch.allclose(mean.double().cpu(), mu, atol=1e-5, rtol=1e-5)
    assert torch.allclose(rstd.double().cpu(), 1.0 / torch.sqrt(var + 1e-5), rtol=1e-4)
    assert torch.allclose(y.permute(0, 3, 1, 2).double().cpu(), ref, atol=1e-4)


@pytest.mark.parametrize("n,H,W", [(2, 64, 96), (1, 48, 80), (1, 96, 144)])
def test_conv2_up4_vs_torch(gpu, n, H, W):
    """head.conv2 by bilinear phases == conv2(cat[interpolate(L, x4), G]) in fp64
    (DeteNet.py:109-112), including the border lines and the IN statistics.
    Ragged sizes: low-res grids that do not fill the 8x16 phase patches."""
    from posfeat_amd import ops
    g = torch.Generator().manual_seed(H * 7 + W)
    h, w = H // 4, W // 4
    L = torch.randn(n, 192, h, w, generator=g)
    G = torch.randn(n, 64, H, W, generator=g)
    wt = torch.randn(128, 256, 3, 3, generator=g) * (2.0 / (256 * 9)) ** 0.5
    b = torch.randn(128, generator=g) * 0.1
    up = F.interpolate(L.double(), size=(H, W), mode="bilinear", align_corners=False)
    ref = F.conv2d(torch.cat([up, G.double()], 1), wt.double(), b.double(), padding=1)
    bound = F.conv2d(torch.cat([up.abs(), G.double().abs()], 1), wt.double().abs(), padding=1)
    wp, bp = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    Ld = L.permute(0, 2, 3, 1).contiguous().to(gpu)
    Gd = G.permute(0, 2, 3, 1).contiguous().to(gpu)
    y, mean, rstd = ops.conv2_up4_instnorm_stats(Ld, Gd, wp, bp)
    torch.cuda.synchronize()
    got = y.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs()
    tol = 4e-6 * bound + 1e-6
    assert torch.all(err <= tol), "max err %g at %s" % (err.max(), (err / tol).argmax())
    mu = ref.mean((2, 3))
    var = ref.var((2, 3), unbiased=False)
    assert torch.allclose(mean.double().cpu(), mu, atol=1e-5, rtol=1e-5)
    assert torch.allclose(rstd.double().cpu(), 1.0 / torch.sqrt(var + 1e-5), rtol=1e-4)
    again, _, _ = ops.conv2_up4_instnorm_stats(Ld, Gd, wp, bp)
    assert torch.equal(y, again)


def test_conv_deterministic(gpu):
    from posfeat_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 64, 96, 128, generator=g).permute(0, 2, 3, 1).contiguous().to(gpu)
    wt = torch.randn(128, 64, 3, 3, generator=g).to(gpu)
    wp, bp = ops.pack_conv_weight(wt)
    a = ops.conv2d_nhwc(x, wp, bp, 128, 3, 3)
    b = ops.conv2d_nhwc(x, wp, bp, 128, 3, 3)
    assert torch.equal(a, b)


def test_layout_roundtrip(gpu):
    from posfeat_amd import ops
    x = torch.randn(2, 40, 13, 17, device=gpu)
    y = ops.nchw_to_nhwc(x, cstride=44)
    assert torch.equal(y[..., :40], x.permute(0, 2, 3, 1))
    assert torch.all(y[..., 40:] == 0)
    z = ops.nhwc_to_nchw(y, c=40)
    assert torch.equal(z, x)
    # whole 64 x 64 tiles (the 16-B transpose: 128 channels, 32 x 48 pixels,
    # channel stride 132) and 3 -> 4 channels (the image's NHWC4 layout)
    x = torch.randn(2, 128, 32, 48, device=gpu)
    y = ops.nchw_to_nhwc(x, cstride=132)
    assert torch.equal(y[..., :128], x.permute(0, 2, 3, 1))
    assert torch.equal(ops.nhwc_to_nchw(y, c=128), x)
    x = torch.randn(3, 3, 16, 24, device=gpu)
    y = ops.nchw_to_nhwc(x, cstride=4)
    assert torch.equal(y[..., :3], x.permute(0, 2, 3, 1))
    assert torch.all(y[..., 3] == 0)


# ------------------------------------------------------------------ detector
def _check_det(gpu, km_np, prefix, d, r, n, un, thr, tm):
    from posfeat_amd import ops
    km = torch.from_numpy(km_np).to(gpu)
    idx, coord, score, counts, nsel = ops.detect(km, r, n, use_nms=un, thr=thr, thr_mod=tm)
    ref_idx = d[prefix + "_idx"][0]
    ref_masked = d[prefix + "_masked"][0]
    assert nsel == ref_idx.shape[0]
    assert int(counts[0].item()) == int(d[prefix + "_count"][0])
    idx = idx[0].cpu().numpy()
    coord = coord[0].cpu().numpy()
    score = score[0].cpu().numpy()
    pos = ref_masked > 0  # zero-score fill rows are compared by count only
    np.testing.assert_array_equal(idx[pos], ref_idx[pos])
    np.testing.assert_array_equal(score[pos], d[prefix + "_kp_score"][0][pos])
    np.testing.assert_allclose(coord[pos], d[prefix + "_coord_n"][0][pos], atol=1e-5, rtol=0)


def test_detector_golden_random(gpu):
    d = np.load(os.path.join(GOLDEN, "detector.npz"))
    from golden_cfg import DET_CONFIGS
    for s in range(3):
        km = np.random.RandomState(s).rand(1, 1, 480, 640).astype(np.float32)
        for name, r, n, un, thr, tm in DET_CONFIGS:
            _check_det(gpu, km, "rand%d_%s" % (s, name), d, r, n, un, thr, tm)


def test_detector_golden_crafted(gpu):
    d = np.load(os.path.join(GOLDEN, "detector.npz"))
    for j in range(4):
        km = d["crafted%d_map" % j]
        from golden_cfg import CRAFTED_CONFIGS
        for name, r, n, un, thr, tm in CRAFTED_CONFIGS:
            _check_det(gpu, km, "crafted%d_%s" % (j, name), d, r, n, un, thr, tm)


def test_detector_batch_min_count(gpu):
    """b>1: n = min count over the batch (preprocess_utils.py:256-257)."""
    from posfeat_amd import ops
    from oracle import detect_ref
    km = np.stack([np.random.RandomState(s).rand(1, 120, 160).astype(np.float32)
                   for s in (5, 6, 7)])
    c_ref, s_ref, i_ref = detect_ref.generate_kpts_single(km, 1, 4000, thr=0.9, thr_mod="abs",
                                                          return_idx=True)
    idx, coord, score, counts, n = ops.detect(torch.from_numpy(km).to(gpu), 1, 4000, thr=0.9,
                                              thr_mod="abs")
    assert n == i_ref.shape[1]
    np.testing.assert_array_equal(idx.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(score.cpu().numpy(), s_ref)
    np.testing.assert_allclose(coord.cpu().numpy(), c_ref, atol=1e-5)


def test_detector_each_equals_per_image(gpu):
    """posfeat_detect_each on a batch == the oracle run on every image alone
    (the reference extraction loop, batch 1): per-image n, idx, score, coord;
    and posfeat_sample_desc_each == the batch-1 sampler row for row, zeros
    past each image's n."""
    from posfeat_amd import ops
    from oracle import detect_ref
    # survivor counts differ per image (thresholds bite differently), one
    # image below the 128 raise
    km = np.stack([np.random.RandomState(s).rand(1, 120, 160).astype(np.float32)
                   for s in (5, 6, 7, 8)])
    km[1] *= 0.5
    km[3, 0, :, 40:] = 0.0
    for r, n, thr in ((1, 4000, 0.9), (2, 600, False), (3, 5000, 0.97)):
        idx, coord, score, counts, nsel = ops.detect(torch.from_numpy(km).to(gpu), r, n, thr=thr,
                                                     thr_mod="abs", sync=False, each=True)
        nsel = nsel.cpu().numpy()
        assert len(set(nsel.tolist())) > 1 or r == 2
        fmap = torch.randn(4, 30, 40, 128, device=gpu)
        desc = ops.sample_desc_nhwc(fmap, coord, c=128, n_valid=torch.from_numpy(nsel).to(gpu),
                                    each=True).cpu()
        for i in range(4):
            c_ref, s_ref, i_ref = detect_ref.generate_kpts_single(km[i:i + 1], r, n, thr=thr,
                                                                  thr_mod="abs", return_idx=True)
            k = int(nsel[i])
            assert k == i_ref.shape[1]
            np.testing.assert_array_equal(idx[i, :k].cpu().numpy(), i_ref[0])
            np.testing.assert_array_equal(score[i, :k].cpu().numpy(), s_ref[0])
            np.testing.assert_allclose(coord[i, :k].cpu().numpy(), c_ref[0], atol=1e-5)
            one = ops.sample_desc_nhwc(fmap[i:i + 1].contiguous(), coord[i:i + 1, :k]).cpu()
            # rows of zero-score fill in an all-zero region have NaN coords (0/0
            # soft-argmax, as the reference): NaN == NaN here
            np.testing.assert_array_equal(desc[i, :k].numpy(), one[0].numpy())
            assert torch.all(desc[i, k:] == 0)


def test_detector_many_ties_at_cut(gpu):
    """> 1024 exactly-equal scores straddling the top-k cut (fallback path) and
    the masked-zero fill path (n raised to 128)."""
    from posfeat_amd import ops
    from oracle import detect_ref
    rs = np.random.RandomState(4)
    km = (rs.randint(0, 4, (1, 1, 200, 260)).astype(np.float32) / 3.0).astype(np.float32)
    for r, n, thr in ((1, 2048, False), (1, 5000, False), (3, 300, 0.5), (2, 64, 0.99)):
        c_ref, s_ref, i_ref = detect_ref.generate_kpts_single(km, r, n, thr=thr, thr_mod="abs",
                                                              return_idx=True)
        idx, coord, score, counts, nn = ops.detect(torch.from_numpy(km).to(gpu), r, n, thr=thr,
                                                   thr_mod="abs")
        assert nn == i_ref.shape[1]
        np.testing.assert_array_equal(idx.cpu().numpy(), i_ref)
        np.testing.assert_array_equal(score.cpu().numpy(), s_ref)


# ------------------------------------------------------------------ sampler
def test_sampler_golden(gpu):
    from posfeat_amd import ops
    d = np.load(os.path.join(GOLDEN, "sampler.npz"))
    fmap = np.random.RandomState(11).randn(2, 128, 24, 32).astype(np.float32)
    x = torch.from_numpy(fmap).to(gpu)
    xn = ops.nchw_to_nhwc(x)
    c = torch.from_numpy(d["coords"]).to(gpu)
    for norm, key, tol in ((True, "desc_norm", 1e-5), (False, "desc_raw", 1e-4)):
        out = ops.sample_desc_nhwc(xn, c, normalize=norm).cpu().numpy()
        np.testing.assert_allclose(out, d[key], atol=tol, rtol=0)
