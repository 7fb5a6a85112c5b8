"""Round-6 engine fusions against their unfused forms (the A/B build, in a
child process):

* POSFEAT_NPFUSE=1 (A/B, off by default) -- head.conv1's instance norm +
  PReLU applied inside the tap GEMM's A loads (conv_bf6x_kernel AM = 4)
  instead of in_apply writing the normalised map: the same arithmetic on the
  same values, so every output is bit-identical;
* POSFEAT_W6STATS -- head.conv1's instance-norm statistics from its F(6x6)
  output transform instead of a pass over its output;
* POSFEAT_NCHWSINK=1 (A/B, off by default) -- conv_fine's epilogue writes
  local_map NCHW too (no layout pass): bit-identical;
* POSFEAT_TAPWS / POSFEAT_WS1X1 / POSFEAT_WSSTEM -- head.conv2's tap GEMM,
  the short-K 1x1 convs and the stem on the weight-stationary kernel vs the
  tuned tiles;
* POSFEAT_DSFUSE -- each stage's first bottleneck conv3 + downsample as one
  two-source GEMM (posfeat_conv1x1_dual) instead of two convs: a different
  fp32 summation order, so the maps agree within tests/tol.py's bounds.
"""
import numpy as np
import pytest
import torch

import tol

pytestmark = pytest.mark.gpu

KEYS = ("local_map", "global_map", "local_map_small", "local_point", "global_feat")

CHILD = """
import os
os.environ[%(var)r] = %(val)r
import numpy as np, torch
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.weights import seeded_state_dicts, seeded_image
bb, hd = seeded_state_dicts(0)
eng = ExtractionEngine(bb, hd, device="cuda:0")
img = torch.stack([torch.from_numpy(seeded_image(s, *%(hw)r)) for s in (4, 5)]).to("cuda:0")
out = eng.run(img)
torch.cuda.synchronize()
np.savez(%(out)r, **{k: out[k].cpu().numpy() for k in %(keys)r})
"""


def _run_default(hw):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_image, seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device="cuda:0")
    img = torch.stack([torch.from_numpy(seeded_image(s, *hw)) for s in (4, 5)]).to("cuda:0")
    out = eng.run(img)
    torch.cuda.synchronize()
    return {k: out[k].cpu().numpy() for k in KEYS}


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_tap_gemm_normalise_on_load_bit_identical(gpu, hw, tmp_path):
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "npfuse_on.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_NPFUSE", val="1", hw=hw, out=out, keys=KEYS), out)
    for k in KEYS:
        assert np.array_equal(got[k], ref[k]), "%s differs (max %g)" % (
            k, np.abs(got[k] - ref[k]).max())


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_conv3_downsample_gemm_vs_two_convs(gpu, hw, tmp_path):
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "dsfuse_off.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_DSFUSE", val="0", hw=hw, out=out, keys=KEYS), out)
    for k in KEYS:
        tol.check(k, torch.from_numpy(got[k]), ref[k], "dsfuse " + k)


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_conv1_stats_from_output_transform(gpu, hw, tmp_path):
    """POSFEAT_W6STATS: head.conv1's instance-norm statistics summed by its
    F(6x6) output transform (fp64 per tile group) vs the statistics pass over
    its output; the backbone maps are untouched (bit-identical), the score map
    within its bound."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "w6stats_off.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_W6STATS", val="0", hw=hw, out=out, keys=KEYS), out)
    for k in ("local_map", "global_map", "local_map_small", "global_feat"):
        assert np.array_equal(got[k], ref[k]), k
    tol.check("local_point", torch.from_numpy(got["local_point"]), ref["local_point"],
              "w6stats local_point")


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_local_map_nchw_from_conv_fine_epilogue(gpu, hw, tmp_path):
    """POSFEAT_NCHWSINK=1: conv_fine's epilogue writes local_map NCHW as well
    (the same bias + ELU on the same tile values) instead of the layout pass
    over its NHWC output: every output bit-identical."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "nchwsink_on.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_NCHWSINK", val="1", hw=hw, out=out, keys=KEYS), out)
    for k in KEYS:
        assert np.array_equal(got[k], ref[k]), "%s differs (max %g)" % (
            k, np.abs(got[k] - ref[k]).max())


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_tap_gemm_weight_stationary(gpu, hw, tmp_path):
    """POSFEAT_TAPWS (default on): head.conv2's tap GEMM on the persistent
    weight-stationary kernel (gemm_ws_kernel: the bf6x tile's six bf16
    terms in the same k order) vs the engine's tuned bf6x tile (A/B
    POSFEAT_TAPWS=0): the backbone maps bit-identical, the score map within
    its bound (bit-identical where the tuned tile is the 128 x 128 bf6x tile
    without split-K)."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "tapws_off.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_TAPWS", val="0", hw=hw, out=out, keys=KEYS), out)
    for k in ("local_map", "global_map", "local_map_small", "global_feat"):
        assert np.array_equal(got[k], ref[k]), k
    tol.check("local_point", torch.from_numpy(got["local_point"]), ref["local_point"],
              "tapws local_point")


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_short_k_1x1_weight_stationary(gpu, hw, tmp_path):
    """POSFEAT_WS1X1: dense 1x1 convs on the weight-stationary kernel with
    bias + residual + activation from registers (A/B =1: every K = 64 / 128 /
    256 conv -- bottleneck conv1 / conv3 with the residual add, conv_fine; the
    default: layer1's N = 64 conv1) vs the tuned bf6x tiles (=0): the same six
    bf16 terms per product in a tile's k order, so every map within its bound
    (measured bit-identical, r16zh)."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "ws1x1_off.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_WS1X1", val="0", hw=hw, out=out, keys=KEYS), out)
    out1 = str(tmp_path / "ws1x1_all.npz")
    every = run_ab_child(CHILD % dict(var="POSFEAT_WS1X1", val="1", hw=hw, out=out1, keys=KEYS), out1)
    for k in KEYS:
        tol.check(k, torch.from_numpy(got[k]), ref[k], "ws1x1 " + k)
        tol.check(k, torch.from_numpy(every[k]), ref[k], "ws1x1=1 " + k)
        print("ws1x1=1", hw, k, float(np.abs(every[k] - ref[k]).max()))
        print("ws1x1", hw, k, float(np.abs(got[k] - ref[k]).max()))


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
def test_stem_weight_stationary(gpu, hw, tmp_path):
    """POSFEAT_WSSTEM=1 (A/B, off by default: slower): the 7x7
    stem on the weight-stationary kernel with the G4 gather (the tap order of
    conv_bf6x_kernel's G4 tile, an eighth all-zero chunk) vs the G4 bf6x
    tile: the same sums, so every map bit-identical."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / "wsstem_on.npz")
    ref = run_ab_child(CHILD % dict(var="POSFEAT_WSSTEM", val="1", hw=hw, out=out, keys=KEYS), out)
    for k in KEYS:
        assert np.array_equal(got[k], ref[k]), "%s differs (max %g)" % (
            k, np.abs(got[k] - ref[k]).max())


@pytest.mark.parametrize("hw", [(128, 160), (96, 224)])
@pytest.mark.parametrize("mode", ["0", "1"])
def test_head_conv1_gemm_weight_stationary(gpu, hw, mode, tmp_path):
    """POSFEAT_WSB (default 3): the batched F(6x6) transform-domain GEMMs of
    head.conv1 (K = N = 192, 96-column tiles) and of layer2 / layer3's conv2
    (K = 128 / 256) on the weight-stationary kernel (grid.y = the transform
    point) vs the bf6x tiles (=0) and vs head.conv1's alone (=1): the same six
    bf16 terms per product in the same k order, so every map within its bound
    (measured bit-identical, r16zz3 / r16zz4)."""
    from conftest import run_ab_child
    got = _run_default(hw)
    out = str(tmp_path / ("wsb_%s.npz" % mode))
    ref = run_ab_child(CHILD % dict(var="POSFEAT_WSB", val=mode, hw=hw, out=out, keys=KEYS), out)
    for k in KEYS:
        tol.check(k, torch.from_numpy(got[k]), ref[k], "wsb " + k)
        print("wsb", mode, hw, k, float(np.abs(got[k] - ref[k]).max()),
              bool(np.array_equal(got[k], ref[k])))
