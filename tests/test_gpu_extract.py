"""extract.py end to end (managers/extractor.py:318-382 drop-in) on the
reference's own configs, checked file by file against the oracle with the
near-tie rule (tests/extract_check.py): no positional slack.

* configs/extract_synthetic.yaml (seeded images, inline model config);
* configs/extract_hpatches.yaml -- BASELINE configs[0]'s entry point -- on a
  one-sequence HPatches-layout tree with a seeded checkpoint directory;
* configs/extract_aachen.yaml on an Aachen-layout tree with db/ and query/
  images: the query images must use ``detector_config_query``
  (/root/reference/managers/extractor.py:335-340);
* the pipelined loop against the reference's serial loop: bit-equal files when
  the batch composition is the same (group 1), oracle-checked when it is not.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import yaml

from conftest import ROOT

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(ROOT, "tools"))

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
    m = networks.PoSFeat(MODEL_CONFIG, torch.device("cuda"))   # seeded weights (seed 0)
    m.set_eval()
    return m


def run_extract(cfg, cwd, env=None):
    p = os.path.join(str(cwd), "cfg_%s.yaml" % cfg["output_root"].replace("/", "_"))
    yaml.safe_dump(cfg, open(p, "w"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "extract.py"), "--config", p],
                       cwd=str(cwd), capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    return os.path.join(str(cwd), "ckpts", cfg["output_root"])


def gpu_maps(model, ims, group=32):
    """local_point of every image under the pipelined loop's batch composition
    (buckets by shape in loader order, at most ``group`` per batch)."""
    out, buckets = {}, {}
    order = []
    for name, x in ims:
        buckets.setdefault(tuple(x.shape), []).append((name, x))
        order.append(name)
    for items in buckets.values():
        for k in range(0, len(items), group):
            chunk = items[k:k + group]
            lp = model.extract(torch.stack([x for _, x in chunk]).cuda())["local_point"]
            for i, (name, _) in enumerate(chunk):
                out[name] = lp[i, 0].cpu().numpy()
    return out


def check_tree(desc_root, postfix, ims, det_cfg_of, model, group=32):
    """Every image's file against the oracle (near-tie aware)."""
    from extract_check import check_file
    from oracle import detect_ref, model_ref
    from posfeat_amd.weights import seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    S_gpu = gpu_maps(model, ims, group)
    stats = []
    for name, x in ims:
        z = np.load(os.path.join(desc_root, name + "." + postfix))
        o = model_ref.posfeat_extract(bb, hd, x[None])
        S_ref = o["local_point"].numpy()
        h, w = x.shape[1:]
        cfg = det_cfg_of(name)
        ref = detect_ref.process_image(S_ref, o["local_map"].numpy(), cfg, h, w)
        delta = float(np.abs(S_gpu[name] - S_ref[0, 0]).max())
        stats.append(check_file(z, ref, S_ref[0, 0], delta, cfg, h, w, tag=name))
    return stats


def test_extract_cli_synthetic(gpu, tmp_path, model):
    """configs/extract_synthetic.yaml: files in the reference format, equal to
    the oracle's Extractor.process up to near-ties."""
    from posfeat_amd.datasets import SyntheticImages
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    cfg["data_config_extract"].update(num_images=3, height=128, width=160)
    cfg["detector_config"]["num_pts"] = 512
    root = run_extract(cfg, tmp_path)
    desc = os.path.join(root, "desc")
    assert sorted(os.listdir(os.path.join(desc, "synthetic"))) == [
        "0000%d.ppm.PoSFeat_seeded" % i for i in range(3)]
    ds = SyntheticImages(cfg["data_config_extract"])
    ims = [(ds[i]["name1"], ds[i]["im1"]) for i in range(3)]
    stats = check_tree(desc, cfg["postfix"], ims, lambda n: cfg["detector_config"], model)
    assert all(nf == 512 for _, nf, _ in stats)
    names = open(os.path.join(root, "image", "name_list.txt")).read().splitlines()
    assert names == ["%d synthetic/%05d.ppm" % (i, i) for i in range(3)]


def test_extract_hpatches_config(gpu, tmp_path, model):
    """configs[0]'s entry point: extract.py --config configs/extract_hpatches.yaml
    (batch 1, num_pts 8192, r 1, thr 0.9 abs; model_config merged from the
    checkpoint directory's config.yaml) on a one-sequence HPatches tree."""
    import extract_e2e
    from posfeat_amd.datasets import HPatch_SIFT
    extract_e2e.make_dataset(str(tmp_path), 1, [(128, 160)])
    extract_e2e.make_checkpoint(str(tmp_path))
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_hpatches.yaml")))
    cfg["data_config_extract"]["data_path"] = str(tmp_path / "data" / "hpatches-sequences-release")
    root = run_extract(cfg, tmp_path)
    desc = os.path.join(root, "desc")
    assert sorted(os.listdir(os.path.join(desc, "v_synth00"))) == [
        "%d.ppm.PoSFeat_mytrain" % i for i in range(1, 7)]
    ds = HPatch_SIFT(cfg["data_config_extract"])
    ims = [(ds[i]["name1"], ds[i]["im1"]) for i in range(len(ds))]
    stats = check_tree(desc, cfg["postfix"], ims, lambda n: cfg["detector_config"], model)
    # 128x160 images hold fewer than 8192 peaks: n = the image's own count
    assert all(nf < 8192 for _, nf, _ in stats)
    names = open(os.path.join(root, "image", "name_list.txt")).read().splitlines()
    assert names == ["%d v_synth00/%d.ppm" % (i, i + 1) for i in range(6)]


def _write_aachen(root, n_db=2, n_query=2, hw=(128, 160)):
    from PIL import Image
    rs = np.random.RandomState(7)
    paths = []
    for sub, n in (("db", n_db), (os.path.join("query", "day", "nexus5x"), n_query)):
        d = os.path.join(root, sub)
        os.makedirs(d, exist_ok=True)
        for i in range(n):
            im = rs.randint(0, 256, (hw[0] // 8, hw[1] // 8, 3)).astype(np.uint8)
            im = Image.fromarray(im).resize((hw[1], hw[0]), Image.BILINEAR)
            p = os.path.join(d, "%d.jpg" % i)
            im.save(p, quality=95)
            paths.append(p)
    return paths


def test_extract_aachen_query_branch(gpu, tmp_path, model):
    """configs/extract_aachen.yaml on db/ + query/*/*/ images: names as the
    reference's Aachen dataset makes them, and the query images detected with
    detector_config_query (set apart here: r 1, thr 0.1, 150 points -- at
    128 x 160 ~200 survivors, so n = 150 exactly) while db images
    keep detector_config (r 3, thr 0.5, 20480)."""
    import extract_e2e
    from posfeat_amd.datasets import Aachen_Day_Night
    data = tmp_path / "aachen"
    _write_aachen(str(data))
    extract_e2e.make_checkpoint(str(tmp_path))
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_aachen.yaml")))
    cfg["data_config_extract"]["data_path"] = str(data)
    cfg["detector_config_query"].update(nms_radius=1, thr=0.1, num_pts=150)
    root = run_extract(cfg, tmp_path)
    desc = os.path.join(root, "desc")
    ds = Aachen_Day_Night(cfg["data_config_extract"])
    ims = [(ds[i]["name1"], ds[i]["im1"]) for i in range(len(ds))]
    assert sorted(n for n, _ in ims) == ["db/0.jpg", "db/1.jpg", "query/day/nexus5x/0.jpg",
                                         "query/day/nexus5x/1.jpg"]

    def det_cfg_of(name):
        return cfg["detector_config_query"] if name.startswith("query/") else \
            cfg["detector_config"]
    stats = check_tree(desc, cfg["postfix"], ims, det_cfg_of, model)
    for (name, _), (_, nf, _) in zip(ims, stats):
        if name.startswith("query/"):
            assert nf == 150, (name, nf)
        else:   # r 3 / thr 0.5: ~75 survivors, n raised to 128 (zero-score fillers)
            assert nf == 128, (name, nf)


@pytest.mark.parametrize("group", ["1", "3"])
def test_extract_pipelined_vs_serial(gpu, tmp_path, model, group):
    """The pipelined loop (shape buckets, uint8 upload + device normalisation,
    async D2H, writer threads) against the reference's serial loop
    (POSFEAT_EXTRACT_PIPELINE=0).  group 1: the same batch composition (B = 1)
    -> bit-equal files.  group 3 (batches of 3 + 2 images): both trees checked
    against the oracle with the near-tie rule."""
    from posfeat_amd.datasets import SyntheticImages
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    cfg["data_config_extract"].update(num_images=5, height=96, width=128, workers=2)
    cfg["detector_config"]["num_pts"] = 300
    roots = {}
    for mode in ("1", "0"):
        cfg["output_root"] = "syn_%s_g%s" % (mode, group)
        roots[mode] = run_extract(cfg, tmp_path, env=dict(POSFEAT_EXTRACT_PIPELINE=mode,
                                                          POSFEAT_EXTRACT_GROUP=group))
        names = open(os.path.join(roots[mode], "image", "name_list.txt")).read().splitlines()
        assert names == ["%d synthetic/%05d.ppm" % (i, i) for i in range(5)]
    files = {m: sorted(os.listdir(os.path.join(r, "desc", "synthetic"))) for m, r in roots.items()}
    assert files["1"] == files["0"] and len(files["1"]) == 5
    if group == "1":
        for f in files["1"]:
            a = np.load(os.path.join(roots["1"], "desc", "synthetic", f))
            b = np.load(os.path.join(roots["0"], "desc", "synthetic", f))
            for k in ("keypoints", "scores", "descriptors"):
                assert np.array_equal(a[k], b[k]), (f, k)
        return
    ds = SyntheticImages(cfg["data_config_extract"])
    ims = [(ds[i]["name1"], ds[i]["im1"]) for i in range(5)]
    check_tree(os.path.join(roots["1"], "desc"), cfg["postfix"], ims,
               lambda n: cfg["detector_config"], model, group=3)
    check_tree(os.path.join(roots["0"], "desc"), cfg["postfix"], ims,
               lambda n: cfg["detector_config"], model, group=1)


def test_extract_many_shapes_bounded_hold(gpu, tmp_path):
    """Many image sizes (HPatches crops each image to /16, Aachen/ETH keep full
    resolution): the shape buckets never fill, and without a bound the pipelined
    loop held the whole stream until the end.  With
    POSFEAT_EXTRACT_HOLD the fullest bucket launches early: at most HOLD images
    wait, every image is written once, in loader order in name_list.txt, with
    its own size's keypoint count."""
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    sizes = [[64, 96], [80, 96], [64, 112], [96, 96], [80, 112], [64, 128]]
    cfg["data_config_extract"].update(num_images=18, sizes=sizes, workers=2)
    cfg["detector_config"]["num_pts"] = 200
    cfg["output_root"] = "syn_shapes"
    root = run_extract(cfg, tmp_path, env=dict(POSFEAT_EXTRACT_GROUP="4",
                                               POSFEAT_EXTRACT_HOLD="5"))
    names = open(os.path.join(root, "image", "name_list.txt")).read().splitlines()
    assert names == ["%d synthetic/%05d.ppm" % (i, i) for i in range(18)]
    files = sorted(os.listdir(os.path.join(root, "desc", "synthetic")))
    assert len(files) == 18
    for f in files:
        z = np.load(os.path.join(root, "desc", "synthetic", f))
        assert z["keypoints"].shape == (200, 2) and z["descriptors"].shape == (200, 128)
    log = open(os.path.join(root, "logging_file.txt")).read()
    held = [int(l.split("at most ")[1].split()[0]) for l in log.splitlines() if "at most" in l]
    assert held and held[-1] <= 5, held
