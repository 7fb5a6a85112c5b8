"""The bf16x6 product arithmetic (posfeat_set_conv_precision(1), the default)
is fp32-accurate: against an fp64 reference its error is no larger than the
fp32-input MFMA's own (mode 0), on the conv shapes it serves (1x1, strided
3x3, the 3x3 stride-1 halo tiles, split-K, the batched Winograd GEMMs) and
through the whole model.

Each fp32 operand is split exactly into three bf16 terms and the six
products of order >= 2^-16 are accumulated in fp32: the per-product error is
~2e-8 relative (3 x 2^-27), below one fp32 rounding (2^-24 ~ 6e-8); the
accumulation is the same kind of fp32 chain.  The bound asserted here:
max|y_bf6 - y64| <= 1.25 max|y_fp32 - y64| + 1e-7 Σ|x||w| per conv, and the
results must differ from mode 0 (the bf16 path really ran)."""
import numpy as np
import pytest
import torch

import tol

pytestmark = pytest.mark.gpu


@pytest.fixture
def precision():
    from posfeat_amd._lib import lib
    prev = lib().posfeat_set_conv_precision(1)
    yield lambda m: lib().posfeat_set_conv_precision(m)
    lib().posfeat_set_conv_precision(prev)


CASES = [  # n, h, w, cin, cout, k, stride, split
    (2, 40, 48, 512, 256, 1, 1, False),
    (2, 40, 48, 256, 64, 1, 1, False),
    (1, 48, 64, 512, 256, 3, 2, False),
    (1, 30, 40, 1024, 256, 1, 1, True),
    (2, 40, 48, 256, 128, 3, 1, False),   # 3x3 stride 1: the halo kernel (H8x128)
    (1, 32, 64, 128, 64, 3, 1, False),    # ... H8x64
    (2, 30, 40, 256, 256, 3, 1, True),    # ... split-K
]


@pytest.mark.parametrize("case", CASES)
def test_bf6_conv_error_le_fp32(gpu, precision, case):
    from posfeat_amd import ops
    n, h, w, cin, cout, k, stride, split = case
    g = torch.Generator().manual_seed(cin + cout + k)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / np.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g) * 0.1
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), stride=stride,
                                     padding=(k - 1) // 2).permute(0, 2, 3, 1)
    mag = torch.nn.functional.conv2d(x.double().abs(), wt.double().abs(), None, stride=stride,
                                     padding=(k - 1) // 2).permute(0, 2, 3, 1)
    xg = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp, bb = ops.pack_conv_weight(wt.to(gpu), b.to(gpu))
    outs = {}
    for mode in (0, 1):
        precision(mode)
        outs[mode] = ops.conv2d_nhwc(xg, wp, bb, cout, k, k, stride=stride,
                                     allow_split=split).cpu().double()
    e32 = float((outs[0] - ref).abs().max())
    e6 = float((outs[1] - ref).abs().max())
    assert not torch.equal(outs[0], outs[1]), "bf16x6 path did not run"
    print("case", case, "fp32 err %.3e  bf16x6 err %.3e  scale %.3e" % (e32, e6, float(mag.max())))
    assert e6 <= 1.25 * e32 + 1e-7 * float(mag.max()), (e6, e32)
    assert e6 <= 2e-6 * float(mag.max())


def test_bf6_winograd_gemm_and_model(gpu, precision):
    """The decoder's batched Winograd GEMMs and the whole extraction model:
    mode 1 vs mode 0 within the fp32 noise of the model (1e-5 of the map
    scale), and mode 1's error vs the torch-CPU oracle of the same order as
    mode 0's (both are fp32 rounding noise of different summation orders)
    and within the parity bounds of tests/tol.py."""
    from oracle import model_ref
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_image, seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    img = torch.from_numpy(seeded_image(4, 96, 128))[None]
    res = {}
    for mode in (0, 1):
        precision(mode)
        eng = ExtractionEngine(bb, hd, device=gpu)
        o = eng.run(img.to(gpu))
        res[mode] = {k: o[k].cpu().double() for k in ("local_point", "local_map", "global_map")}
        eng.close()
    ref = model_ref.posfeat_extract(bb, hd, img)
    for k in ("local_point", "local_map", "global_map"):
        s = max(1.0, float(ref[k].abs().max()))
        d01 = float((res[0][k] - res[1][k]).abs().max())
        e0 = float((res[0][k] - ref[k].double()).abs().max())
        e1 = float((res[1][k] - ref[k].double()).abs().max())
        assert d01 <= 1e-5 * s, (k, d01)
        assert e1 <= 2 * e0 + 1e-6 * s, (k, e1, e0)
        tol.check(k, res[1][k], ref[k], "bf16x6 model vs oracle")
