"""GPU tests of the drop-in Python surfaces (networks.PoSFeat, losses.
preprocess_utils, managers.extractor.Extractor, extract.py) -- each checked
against the oracle / golden vectors."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import tol

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

MODEL_CONFIG = {
    "backbone": "ResUNet",
    "backbone_config": {"encoder": "resnet50", "pretrained": True, "coarse_out_ch": 128,
                        "fine_out_ch": 128},
    "localheader": "KeypointDet",
    "localheader_config": {"in_channels": 192, "prior": "identity", "act": "Softplus"},
    "align_local_grad": False,
    "local_input_elements": ["local_map", "local_map_small"],
    "local_with_img": True,
}


@pytest.fixture(scope="module")
def model():
    from posfeat_amd import networks
    m = networks.PoSFeat(MODEL_CONFIG, torch.device("cuda"))
    m.set_eval()
    return m


def test_posfeat_extract_matches_golden(gpu, model):
    from posfeat_amd.weights import seeded_image
    d = np.load(os.path.join(GOLDEN, "model_small.npz"))
    img = torch.from_numpy(seeded_image(0, 96, 128))[None].to(gpu)
    out = model.extract(img)
    assert set(out.keys()) == {"local_map", "global_map", "global_feat", "local_point",
                               "local_thr", "global_point"}
    assert out["local_thr"].abs().sum() == 0 and out["global_point"].shape == (1, 1, 6, 8)
    for k in ("local_map", "global_map", "local_point", "global_feat"):
        tol.check(k, out[k], d["a_" + k], "PoSFeat.extract vs golden")


def test_checkpoint_roundtrip(gpu, model, tmp_path):
    from posfeat_amd import networks
    from posfeat_amd.weights import seeded_image, seeded_state_dicts
    bb, hd = seeded_state_dicts(3)
    model2 = networks.PoSFeat(MODEL_CONFIG, torch.device("cuda"))
    model2.backbone.load_state_dict(bb)
    model2.localheader.load_state_dict(hd)
    model2.save_checkpoint(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["backbone.pth", "localheader.pth"]
    model3 = networks.PoSFeat(MODEL_CONFIG, torch.device("cuda"))
    model3.load_checkpoint(str(tmp_path))
    model2.set_eval()
    model3.set_eval()
    img = torch.from_numpy(seeded_image(5, 64, 96))[None].to(gpu)
    a = model2.extract(img)["local_point"]
    b = model3.extract(img)["local_point"]
    assert torch.equal(a, b)
    c = model.extract(img)["local_point"]   # different weights -> different map
    assert not torch.equal(a, c)
    # DDP-prefixed checkpoints load too
    sd = {"module." + k: v for k, v in torch.load(tmp_path / "backbone.pth").items()}
    torch.save(sd, tmp_path / "backbone.pth")
    model3.load_checkpoint(str(tmp_path))
    assert torch.equal(model3.extract(img)["local_point"], a)


def test_resunet_forward(gpu, model):
    from oracle import model_ref
    from posfeat_amd.weights import seeded_image
    img = torch.from_numpy(seeded_image(2, 64, 96))[None]
    out = model.backbone(img.to(gpu))
    ref = model_ref.resunet_forward({k: v.cpu() for k, v in model.backbone.state_dict().items()}, img)
    for k in ("global_map", "local_map", "local_map_small"):
        tol.check(k, out[k], ref[k], "ResUNet.forward vs oracle")


def test_keypointdet_forward_standalone(gpu, model):
    """KeypointDet.forward([x, img]) on its own (DeteNet.py:102-121; the engine's
    head-only mode): x = cat[local_map, local_map_small] of the REFERENCE's
    backbone run (golden), so the head is checked against the reference head."""
    from posfeat_amd.weights import seeded_image
    d = np.load(os.path.join(GOLDEN, "model_small.npz"))
    for tag, hw, seed in (("a", (96, 128), 0), ("b", (64, 96), 1)):
        img = torch.from_numpy(seeded_image(seed, *hw))[None].to(gpu)
        x = torch.from_numpy(np.concatenate([d[tag + "_local_map"], d[tag + "_local_map_small"]],
                                            1)).to(gpu)
        lp = model.localheader([x, img])
        ref = d[tag + "_local_point"]
        assert lp.shape == ref.shape
        tol.check("local_point", lp, ref, "KeypointDet.forward %s vs golden" % tag)
    # and it equals the fused PoSFeat.extract path on the same inputs
    img = torch.from_numpy(seeded_image(3, 96, 128))[None].to(gpu)
    full = model.extract(img)
    bbo = model.backbone(img)
    x = torch.cat([bbo["local_map"], bbo["local_map_small"]], 1)
    lp = model.localheader([x, img])
    assert (lp - full["local_point"]).abs().max().item() <= 1e-5 * max(
        1.0, full["local_point"].abs().max().item())


def test_preprocess_utils_dropins(gpu):
    from oracle import detect_ref
    from posfeat_amd.losses import preprocess_utils as pu
    km = np.random.RandomState(9).rand(2, 1, 96, 128).astype(np.float32)
    coord, score = pu.generate_kpts_single(torch.from_numpy(km).to(gpu), 1, 300, thr=0.9,
                                           thr_mod="abs")
    c_ref, s_ref = detect_ref.generate_kpts_single(km, 1, 300, thr=0.9, thr_mod="abs")
    np.testing.assert_array_equal(score.cpu().numpy(), s_ref)
    np.testing.assert_allclose(coord.cpu().numpy(), c_ref, atol=1e-5)
    d = np.load(os.path.join(GOLDEN, "detector.npz"))
    for j in range(4):
        m = d["crafted%d_map" % j]
        for r in (1, 2, 3):
            got = pu.nms(torch.from_numpy(m).to(gpu), r)[0, 0].cpu().numpy()
            np.testing.assert_array_equal(got, detect_ref.nms(m[0, 0], r))
    s = np.load(os.path.join(GOLDEN, "sampler.npz"))
    fmap = torch.from_numpy(np.random.RandomState(11).randn(2, 128, 24, 32).astype(np.float32))
    desc = pu.sample_feat_by_coord(fmap.to(gpu), torch.from_numpy(s["coords"]).to(gpu), True)
    np.testing.assert_allclose(desc.cpu().numpy(), s["desc_norm"], atol=1e-5)
    with pytest.raises(NotImplementedError):
        pu.generate_kpts_single(torch.from_numpy(km).to(gpu), 1, 300, stable=False)
    # the async form (Extractor's pipelined loop) reports the reference's n,
    # including the raise to 128 when fewer points survive NMS + threshold
    small = np.random.RandomState(4).rand(1, 1, 40, 48).astype(np.float32)
    for r, npts in ((3, 20480), (1, 50), (1, 20000)):
        c_s, s_s = pu.generate_kpts_single(torch.from_numpy(small).to(gpu), r, npts, thr=0.5,
                                           thr_mod="abs")
        c_a, s_a, n_a = pu.generate_kpts_single_async(torch.from_numpy(small).to(gpu), r, npts,
                                                      thr=0.5, thr_mod="abs")
        n = int(n_a[0])
        assert n == c_s.shape[1], (r, npts, n, c_s.shape)
        assert torch.equal(c_a[:, :n], c_s) and torch.equal(s_a[:, :n], s_s)
        c_r, _ = detect_ref.generate_kpts_single(small, r, npts, thr=0.5, thr_mod="abs")
        assert c_r.shape[1] == n


def test_normalize_rgb8_bit_exact(gpu):
    """The device input transform equals datasets.to_input's host result bit for bit."""
    from posfeat_amd import ops
    from posfeat_amd.datasets import to_input
    rs = np.random.RandomState(3)
    im = rs.randint(0, 256, (2, 50, 70, 3)).astype(np.uint8)
    im[0, 0, :3] = [[0, 0, 0], [255, 255, 255], [128, 1, 254]]
    got = ops.normalize_rgb8(torch.from_numpy(im).to(gpu)).cpu()
    for i in range(2):
        ref, _ = to_input(im[i])                  # crops 50x70 to 48x64
        assert torch.equal(got[i, :, :48, :64], ref)
