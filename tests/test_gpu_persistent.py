"""The persistent pre-split-weight GEMM tiles (conv_bf6p_kernel,
posfeat_set_conv_persistent(1), an A/B mode) against one workgroup per tile
(conv_bf6b_kernel, mode 0, the default): same products in the same order and the same
epilogue arithmetic, so every engine output is bit-identical.  The dense
GEMMs it serves are the decoder / encoder Winograd transform-domain GEMMs
(batched over the 36 or 16 transform points), the keypoint head's tap GEMM
(K = 192), the 1x1 layers with bias + ReLU + residual, and the stride-2 1x1
downsample convs -- all of them run in one extraction forward.  The 480x640
B=2 case crosses several tiles per workgroup (the grid is capped at 512);
at 32x64 the layer3 GEMMs have fewer tiles than the eight XCD groups."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def persistent():
    from posfeat_amd._lib import lib
    prev = lib().posfeat_set_conv_persistent(-1)
    yield lambda m: lib().posfeat_set_conv_persistent(m)
    lib().posfeat_set_conv_persistent(prev)


@pytest.mark.parametrize("shape", [(1, 32, 64), (2, 96, 128), (2, 480, 640)])
def test_persistent_tiles_bit_identical(gpu, persistent, shape):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_state_dicts, seeded_image
    b, H, W = shape
    bb, hd = seeded_state_dicts(0)
    imgs = torch.from_numpy(np.stack([seeded_image(30 + i, H, W) for i in range(b)])).to(gpu)
    outs = []
    for mode in (0, 1):
        assert persistent(mode) in (0, 1)
        eng = ExtractionEngine(bb, hd, device=gpu)
        eng.run(imgs)
        o = eng.run(imgs, outputs=("local_map", "global_map", "global_feat"))
        torch.cuda.synchronize()
        outs.append({k: v.detach().cpu().clone() for k, v in o.items() if not k.startswith("_")})
        eng.close()
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
    assert torch.isfinite(outs[1]["local_point"]).all()
