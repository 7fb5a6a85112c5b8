"""The dense pre-split GEMM tiles on v_mfma_f32_16x16x32_bf16
(conv_bf6x_kernel, conv.hip): the 1x1 convs the engine runs with weight
planes, and the batched Winograd GEMMs.

The products are the same six bf16 terms as the 32x32x16 tiles (fp32-exact
per product); only the fp32 accumulation grouping differs,
so the bound is the bf16x6 one of test_gpu_precision.py: against an fp64
reference, no more than 1.25x the fp32-input MFMA's own error (mode 0) plus
1e-7 of sum|x||w|, and <= 2e-6 of sum|x||w|.  Covered: M not a multiple of
the 128-row tile, Cout 64 / 128 / 192 / 1024 (both column tiles, ragged
column tiles), bias + residual + ReLU / ELU epilogues, split-K, K from one
chunk to 32 chunks, and stride-2 1x1 convs (the downsample layers)."""
import os
import subprocess
import sys

import numpy as np

from conftest import ab_env
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [  # n, h, w, cin, cout, act, residual, split, stride
    (2, 40, 48, 512, 256, "none", False, False, 1),
    (2, 7, 9, 64, 64, "relu", True, False, 1),        # M = 126 < one tile
    (1, 30, 40, 1024, 256, "relu", True, True, 1),    # layer3 conv1 shape, split-K
    (1, 30, 40, 256, 1024, "relu", True, False, 1),   # layer3 conv3 + residual
    (2, 24, 40, 192, 1152, "none", False, False, 1),  # the tap GEMM's K and N
    (1, 33, 41, 32, 192, "elu", False, False, 1),     # K = one chunk, ragged M, 3 x 64 columns
    (1, 16, 20, 256, 96, "elu", True, False, 1),      # Cout % 64 != 0: ragged column tile
    (2, 60, 80, 512, 1024, "none", False, False, 2),  # layer3.0.downsample (stride 2)
    (1, 31, 41, 256, 128, "relu", True, False, 2),    # stride 2 on odd sizes + residual
    (2, 6, 13, 1152, 192, "none", False, False, 1),   # the tap adjoint's K and N, M = 156
    (1, 12, 13, 576, 192, "none", False, False, 1),   # head.conv1 Winograd GEMM shape
]
TILES = (29, 30, 31)  # TILE_BF6X_128x128, _128x64, _256x128: each legal one, bit-identical


@pytest.fixture
def precision():
    from posfeat_amd._lib import lib
    prev = lib().posfeat_set_conv_precision(1)
    yield lambda m: lib().posfeat_set_conv_precision(m)
    lib().posfeat_set_conv_precision(prev)


@pytest.mark.parametrize("case", CASES)
def test_bf6x_dense_conv_vs_fp64(gpu, precision, case):
    from posfeat_amd import ops
    n, h, w, cin, cout, act, residual, split, stride = case
    g = torch.Generator().manual_seed(7 * cin + cout)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 1, 1, generator=g) / np.sqrt(cin)
    b = torch.randn(cout, generator=g) * 0.1
    oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
    r = torch.randn(n, oh, ow, cout, generator=g) if residual else None
    pre = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(),
                                     stride=stride).permute(0, 2, 3, 1)
    if residual:
        pre = pre + r.double()
    ref = {"none": pre, "relu": pre.clamp_min(0),
           "elu": torch.nn.functional.elu(pre)}[act]
    mag = torch.nn.functional.conv2d(x.double().abs(), wt.double().abs(),
                                     stride=stride).permute(0, 2, 3, 1)
    if residual:
        mag = mag + r.double().abs()
    xg = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp, bb = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    planes = ops.split_weight_planes(wp)
    rg = r.to(gpu) if residual else None
    precision(1)
    y6 = ops.conv2d_nhwc_planes(xg, wp, planes, bb, cout, 1, 1, stride=stride, act=act, res=rg,
                                allow_split=split).cpu().double()
    for t in TILES:   # every tile the autotuner may pick: the same bits
        yt = ops.conv2d_nhwc_planes(xg, wp, planes, bb, cout, 1, 1, stride=stride, act=act,
                                    res=rg, allow_split=split, tile=t).cpu().double()
        assert torch.equal(yt, y6), ("tile", t, float((yt - y6).abs().max()))
    precision(0)
    y32 = ops.conv2d_nhwc(xg, wp, bb, cout, 1, 1, stride=stride, act=act, res=rg).cpu().double()
    torch.cuda.synchronize()
    e32 = float((y32 - ref).abs().max())
    e6 = float((y6 - ref).abs().max())
    scale = float(mag.max())
    print("case", case, "fp32 err %.3e  bf16x6 (16x16x32) err %.3e  scale %.3e" % (e32, e6, scale))
    assert torch.isfinite(y6).all()
    assert e6 <= 1.25 * e32 + 1e-7 * scale, (e6, e32)
    assert e6 <= 2e-6 * scale


CODE = r"""
import sys, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.weights import seeded_image, seeded_state_dicts
bb, hd = seeded_state_dicts(0)
eng = ExtractionEngine(bb, hd, device="cuda:0")
img = torch.from_numpy(np.stack([seeded_image(60 + i, 480, 640) for i in range(4)])).cuda()
r = eng.run(img, outputs=("local_map", "global_map"))
torch.cuda.synchronize()
np.savez(%(out)r, lp=r["local_point"].cpu().numpy(), lm=r["local_map"].cpu().numpy(),
         gm=r["global_map"].cpu().numpy())
"""


def test_bf6x_engine_vs_bf6d(tmp_path):
    """The whole extraction model with the 16x16x32 dense tiles (default) vs
    the 32x32x16 bf6d tiles (POSFEAT_BF6X=0): both fp32-accurate, different
    accumulation grouping -- within 1e-5 of each map's scale, and not
    bit-identical (the 16x16x32 path really ran)."""
    res = {}
    for tag, env in (("x", ab_env()), ("d", dict(ab_env(), POSFEAT_BF6X="0"))):
        out = str(tmp_path / ("%s.npz" % tag))
        subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "out": out}],
                       env=dict(os.environ, **env), check=True, timeout=240)
        res[tag] = np.load(out)
    differ = False
    for k in ("lp", "lm", "gm"):
        a, b = res["x"][k].astype(np.float64), res["d"][k].astype(np.float64)
        s = max(1.0, np.abs(b).max())
        assert np.abs(a - b).max() <= 1e-5 * s, (k, np.abs(a - b).max(), s)
        differ |= not np.array_equal(a, b)
    assert differ, "the 16x16x32 tiles did not run"


def test_bf6x_rb4_bit_identical(tmp_path):
    """The 256-row 16x16x32 tiles (RB = 4: TILE_BF6X_256x128 = 31, forced on
    every dense conv and on the batched Winograd GEMMs) run the same MFMA
    sequence per output element as the 128-row ones: bit-identical engine
    outputs (they are autotune candidates of each other)."""
    res = {}
    for tag, env in (("r2", ab_env()),
                     ("r4", dict(ab_env(), POSFEAT_BF6X_RB4="1", POSFEAT_CONV_TILE="31"))):
        out = str(tmp_path / ("%s.npz" % tag))
        subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "out": out}],
                       env=dict(os.environ, **env), check=True, timeout=240)
        res[tag] = np.load(out)
    for k in ("lp", "lm", "gm"):
        np.testing.assert_array_equal(res["r4"][k], res["r2"][k], err_msg=k)


@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 37, 53), (3, 480, 640)])
def test_bf6x_stem_gather_vs_fp64(gpu, precision, shape):
    """The 7x7 stride-2 stem (4-channel NHWC4 input, K order (kh, kw, c4)) on
    the bf6x tile with per-lane tap gathers (conv_bf6x_kernel G4): against fp64
    within the bf16x6 bound, on even, odd and the metric's image sizes (zero
    padding at every border, the zero fourth channel)."""
    from posfeat_amd import ops
    n, h, w = shape
    g = torch.Generator().manual_seed(h * w)
    x = torch.randn(n, 3, h, w, generator=g)
    wt = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
    b = torch.randn(64, generator=g) * 0.1
    pre = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), stride=2, padding=3)
    ref = pre.clamp_min(0).permute(0, 2, 3, 1)
    mag = torch.nn.functional.conv2d(x.double().abs(), wt.double().abs(), None, stride=2,
                                     padding=3).permute(0, 2, 3, 1)
    x4 = torch.zeros(n, h, w, 4)
    x4[..., :3] = x.permute(0, 2, 3, 1)
    xg = x4.contiguous().to(gpu)
    wp, bb = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    planes = ops.split_weight_planes(wp)
    precision(1)
    y6 = ops.conv2d_nhwc_planes(xg, wp, planes, bb, 64, 7, 7, stride=2, pad=3, act="relu",
                                cin=4).cpu().double()
    precision(0)
    y32 = ops.conv2d_nhwc(xg, wp, bb, 64, 7, 7, stride=2, pad=3, act="relu", cin=4).cpu().double()
    torch.cuda.synchronize()
    e32 = float((y32 - ref).abs().max())
    e6 = float((y6 - ref).abs().max())
    scale = float(mag.max())
    print("stem", shape, "fp32 err %.3e  bf16x6 G4 err %.3e  scale %.3e" % (e32, e6, scale))
    assert e6 <= 1.25 * e32 + 1e-7 * scale, (e6, e32)
    assert e6 <= 2e-6 * scale


GT_CASES = [  # n, h, w, cin, cout, k, stride, act, residual
    (2, 30, 40, 64, 64, 3, 1, "relu", False),     # layer1 conv2 shape (scaled)
    (1, 33, 41, 64, 96, 3, 1, "elu", True),       # ragged M and N, residual
    (2, 30, 40, 128, 128, 3, 2, "relu", False),   # layer2.0 conv2 (stride 2)
    (1, 17, 23, 256, 256, 3, 2, "none", False),   # odd sizes, stride 2
    (1, 12, 20, 512, 128, 3, 1, "none", False),   # K = 144 chunks
]


@pytest.mark.parametrize("case", GT_CASES)
def test_bf6x_slab_tap_gather_vs_fp64(gpu, precision, case):
    """3x3 convs with Cin % 32 == 0 on the bf6x tile's (slab, tap) gather
    (conv_bf6x_kernel GT): against fp64 within the bf16x6 bound, zero padding
    at every border, strides 1 and 2; every legal BF6X tile bit-identical."""
    from posfeat_amd import ops
    n, h, w, cin, cout, k, stride, act, residual = case
    g = torch.Generator().manual_seed(cin * 3 + cout + stride)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / np.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g) * 0.1
    pre = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), stride=stride,
                                     padding=1).permute(0, 2, 3, 1)
    oh, ow = pre.shape[1], pre.shape[2]
    r = torch.randn(n, oh, ow, cout, generator=g) if residual else None
    if residual:
        pre = pre + r.double()
    ref = {"none": pre, "relu": pre.clamp_min(0), "elu": torch.nn.functional.elu(pre)}[act]
    mag = torch.nn.functional.conv2d(x.double().abs(), wt.double().abs(), None, stride=stride,
                                     padding=1).permute(0, 2, 3, 1)
    if residual:
        mag = mag + r.double().abs()
    xg = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp, bb = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    planes = ops.split_weight_planes(wp)
    rg = r.to(gpu) if residual else None
    precision(1)
    y6 = ops.conv2d_nhwc_planes(xg, wp, planes, bb, cout, k, k, stride=stride, act=act,
                                res=rg).cpu().double()
    for t in TILES:
        yt = ops.conv2d_nhwc_planes(xg, wp, planes, bb, cout, k, k, stride=stride, act=act,
                                    res=rg, tile=t).cpu().double()
        assert torch.equal(yt, y6), ("tile", t, float((yt - y6).abs().max()))
    precision(0)
    y32 = ops.conv2d_nhwc(xg, wp, bb, cout, k, k, stride=stride, act=act, res=rg).cpu().double()
    torch.cuda.synchronize()
    e32 = float((y32 - ref).abs().max())
    e6 = float((y6 - ref).abs().max())
    scale = float(mag.max())
    print("gt", case, "fp32 err %.3e  bf16x6 GT err %.3e  scale %.3e" % (e32, e6, scale))
    assert e6 <= 1.25 * e32 + 1e-7 * scale, (e6, e32)
    assert e6 <= 2e-6 * scale
