"""GPU tests of the drop-in Python surfaces (networks.PoSFeat, losses.
preprocess_utils, managers.extractor.Extractor, extract.py) -- each checked
against the oracle / golden vectors."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

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
        ref = d["a_" + k]
        err = np.abs(out[k].cpu().numpy() - ref).max()
        assert err <= 1e-4 * max(1.0, np.abs(ref).max()), k


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
        err = (out[k].cpu() - ref[k]).abs().max().item()
        assert err <= 1e-4 * max(1.0, ref[k].abs().max().item()), k


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
        err = np.abs(lp.cpu().numpy() - ref).max()
        assert err <= 1e-4 * max(1.0, np.abs(ref).max()), (tag, err)
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


def test_extract_cli_synthetic(gpu, tmp_path):
    """extract.py end to end on the synthetic config: npz files in the
    reference format, identical (near-tie aware) to the oracle's process()."""
    import yaml
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    cfg["data_config_extract"].update(num_images=2, height=128, width=160)
    cfg["detector_config"]["num_pts"] = 512
    p = tmp_path / "cfg.yaml"
    yaml.safe_dump(cfg, open(p, "w"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "extract.py"), "--config", str(p)],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out_dir = tmp_path / "ckpts" / cfg["output_root"] / "desc" / "synthetic"
    files = sorted(os.listdir(out_dir))
    assert files == ["00000.ppm.PoSFeat_seeded", "00001.ppm.PoSFeat_seeded"]
    from oracle import model_ref, detect_ref
    from posfeat_amd.datasets import SyntheticImages
    from posfeat_amd.weights import seeded_state_dicts
    from near_tie import explain_differences
    bb, hd = seeded_state_dicts(0)
    ds = SyntheticImages(cfg["data_config_extract"])
    for i, f in enumerate(files):
        z = np.load(out_dir / f)
        assert z["keypoints"].dtype == np.float32 and z["keypoints"].shape[1] == 2
        assert z["scores"].shape == (z["keypoints"].shape[0], 1)
        assert z["descriptors"].shape == (z["keypoints"].shape[0], 128)
        np.testing.assert_allclose(np.linalg.norm(z["descriptors"], axis=1), 1.0, atol=1e-5)
        img = ds[i]["im1"][None]
        o = model_ref.posfeat_extract(bb, hd, img)
        ref = detect_ref.process_image(o["local_point"].numpy(), o["local_map"].numpy(),
                                       cfg["detector_config"], 128, 160)
        assert z["keypoints"].shape[0] == ref["kpt"].shape[0]
        # match keypoints by position: common ones must agree in desc/score
        kp = np.round(z["keypoints"], 3)
        rk = np.round(ref["kpt"], 3)
        common = {tuple(k): j for j, k in enumerate(rk)}
        hit = [(i2, common[tuple(k)]) for i2, k in enumerate(kp) if tuple(k) in common]
        assert len(hit) >= 0.97 * len(kp)
        a, b = np.array(hit).T
        np.testing.assert_allclose(z["descriptors"][a], ref["desc"][0][b], atol=1e-4)
        np.testing.assert_allclose(z["scores"][a], ref["kp_score"][0][b], atol=1e-4)


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


def test_extract_pipelined_equals_serial(gpu, tmp_path):
    """The pipelined loop (same-size grouping, uint8 upload, async D2H, writer
    thread) writes the same files as the reference's serial loop."""
    import yaml
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    cfg["data_config_extract"].update(num_images=5, height=96, width=128, workers=2)
    cfg["detector_config"]["num_pts"] = 300
    outs = {}
    for mode in ("1", "0"):
        cfg["output_root"] = "syn_" + mode
        p = tmp_path / ("cfg%s.yaml" % mode)
        yaml.safe_dump(cfg, open(p, "w"))
        env = dict(os.environ, POSFEAT_EXTRACT_PIPELINE=mode, POSFEAT_EXTRACT_GROUP="3")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "extract.py"), "--config", str(p)],
                           cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        d = tmp_path / "ckpts" / cfg["output_root"] / "desc" / "synthetic"
        outs[mode] = {f: np.load(d / f) for f in sorted(os.listdir(d))}
        names = open(tmp_path / "ckpts" / cfg["output_root"] / "image" / "name_list.txt").read()
        assert names.splitlines()[4] == "4 synthetic/00004.ppm"
    assert list(outs["1"]) == list(outs["0"]) and len(outs["1"]) == 5
    for f in outs["1"]:
        a, b = outs["1"][f], outs["0"][f]
        assert a["keypoints"].shape == b["keypoints"].shape
        ka, kb = np.round(a["keypoints"], 3), np.round(b["keypoints"], 3)
        common = {tuple(k): j for j, k in enumerate(kb)}
        hit = [(i, common[tuple(k)]) for i, k in enumerate(ka) if tuple(k) in common]
        assert len(hit) >= 0.97 * len(ka)
        ia, ib = np.array(hit).T
        np.testing.assert_allclose(a["descriptors"][ia], b["descriptors"][ib], atol=1e-4)
        np.testing.assert_allclose(a["scores"][ia], b["scores"][ib], atol=1e-4)
