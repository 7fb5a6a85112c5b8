"""Generate golden vectors by running the REFERENCE's own Python (build container only).

Run from the repo root:  ``python tests/golden/gen_golden.py``  (needs /root/reference).

What is imported from the reference (unmodified, read-only):
* ``losses`` package (losses/__init__.py: preprocess, preprocess_utils,
  epipolarloss, kploss) -- torch-only, imports cleanly;
* ``networks/DeteNet.py`` (KeypointDet) and ``networks/DescNet.py`` (ResUNet,
  conv, upconv) loaded by file path.  ``networks/__init__.py`` is NOT used
  because PoSFeat_model.py imports the absent ``path`` package.

Third-party pieces that are absent here and restated instead:
* torchvision ``resnet50`` (DescNet.py:25): the ResUNet instance is assembled
  with ``ResUNet.__new__`` and its encoder modules are taken from
  ``oracle/torchvision_resnet.py``; decoder modules are the reference's own
  ``conv``/``upconv`` classes, and ``ResUNet.forward`` is the reference code.
* ``PoSFeat.extract`` glue (PoSFeat_model.py:91-134) is restated inline below
  (cat + detach + [local_input, img] + ones global prior + global_feat).

Outputs (small .npz fixtures, inputs are regenerated from seeds by the tests):
  model_small.npz, detector.npz, sampler.npz, extract_full.npz
"""
import importlib.util
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from posfeat_amd.weights import seeded_state_dicts, seeded_image  # noqa: E402
from oracle.torchvision_resnet import ResNet50Stem  # noqa: E402
import losses as ref_losses  # noqa: E402  (reference package)
from losses import preprocess_utils as ref_putils  # noqa: E402


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ref_desc = _load("ref_DescNet", os.path.join(REF, "networks", "DescNet.py"))
ref_dete = _load("ref_DeteNet", os.path.join(REF, "networks", "DeteNet.py"))


def build_ref_resunet():
    """ResUNet(encoder='resnet50', coarse_out_ch=128, fine_out_ch=128) assembled
    without torchvision; attribute order mirrors DescNet.py:12-48."""
    m = ref_desc.ResUNet.__new__(ref_desc.ResUNet)
    nn.Module.__init__(m)
    r = ResNet50Stem()
    filters = [256, 512, 1024, 2048]
    m.firstconv, m.firstbn, m.firstrelu, m.firstmaxpool = r.conv1, r.bn1, r.relu, r.maxpool
    m.layer1, m.layer2, m.layer3 = r.layer1, r.layer2, r.layer3
    m.conv_coarse = ref_desc.conv(filters[2], 128, 1, 1)
    m.upconv3 = ref_desc.upconv(filters[2], 512, 3, 2)
    m.iconv3 = ref_desc.conv(filters[1] + 512, 512, 3, 1)
    m.upconv2 = ref_desc.upconv(512, 256, 3, 2)
    m.iconv2 = ref_desc.conv(filters[0] + 256, 256, 3, 1)
    m.conv_fine = ref_desc.conv(256, 128, 1, 1)
    m.out_channels = [128, 128]
    return m


def build_ref_models(seed=0):
    bb_sd, hd_sd = seeded_state_dicts(seed)
    bb = build_ref_resunet()
    bb.load_state_dict(bb_sd, strict=True)
    hd = ref_dete.KeypointDet(in_channels=192, out_channels=1, prior="identity", act="Softplus")
    hd.load_state_dict(hd_sd, strict=True)
    bb.eval()
    hd.eval()
    return bb, hd


@torch.no_grad()
def ref_extract(bb, hd, img):
    """Restatement of PoSFeat.extract glue (PoSFeat_model.py:91-134) around the
    reference modules."""
    feat_maps = bb(img)
    b, c, h, w = feat_maps["global_map"].shape
    g_map = torch.ones(b, 1, h, w).type_as(feat_maps["local_map"])
    local_input = torch.cat([feat_maps["local_map"], feat_maps["local_map_small"]], dim=1).detach()
    l_map = hd([local_input, img])
    g_desc = F.normalize(g_map * feat_maps["global_map"], p=2, dim=1).mean([2, 3])
    return {"local_map": feat_maps["local_map"], "global_map": feat_maps["global_map"],
            "local_map_small": feat_maps["local_map_small"], "local_point": l_map,
            "global_feat": g_desc}


@torch.no_grad()
def ref_detect_with_idx(kp_map, nms_radius, num_pts, use_nms=True, thr=False, thr_mod="mean"):
    """Reference generate_kpts_single outputs plus the idx of its line 264
    (recomputed with the reference's own ``nms`` and the same expression), and
    canonicalised to the (score desc, idx asc) tie rule."""
    kps, kp_score = ref_putils.generate_kpts_single(
        kp_map, nms_radius, num_pts, stable=True, use_nms=use_nms, thr=thr, thr_mod=thr_mod)
    b, _, h, w = kp_map.shape
    inner = kp_map[:, :, 1:-1, 1:-1]
    nms_mask = ref_putils.nms(inner, nms_radius) if use_nms else torch.ones_like(inner)
    if thr:
        if thr_mod == "max":
            kp_thr = inner.reshape(b, 1, -1).max(2)[0]
        elif thr_mod == "mean":
            kp_thr = inner.reshape(b, 1, -1).mean(2)
        else:
            kp_thr = torch.tensor(1.).to(kp_map).repeat(b)
        nms_mask = (inner > thr * kp_thr.view(b, 1, 1, 1)) * nms_mask
    count = nms_mask.reshape(b, -1).sum(1)
    n = kps.shape[1]
    masked = (nms_mask * inner).permute(0, 2, 3, 1).contiguous().view(b, -1)
    vals, idx = masked.topk(n)
    # canonicalise runs of equal values: idx ascending
    vals = vals.numpy()
    idx = idx.numpy().copy()
    kps = kps.numpy().copy()
    kp_score = kp_score.numpy().copy()
    for i in range(b):
        order = np.lexsort((idx[i], -vals[i].astype(np.float64)))
        idx[i] = idx[i][order]
        kps[i] = kps[i][order]
        kp_score[i] = kp_score[i][order]
        vals[i] = vals[i][order]
    return {"idx": idx.astype(np.int32), "coord_n": kps.astype(np.float32),
            "kp_score": kp_score.astype(np.float32), "count": count.numpy().astype(np.int64),
            "masked": vals.astype(np.float32)}


def crafted_maps():
    """Small hand-made score maps exercising ties, plateaus, borders (1x1x20x28)."""
    maps = []
    rs = np.random.RandomState(7)
    a = rs.rand(20, 28).astype(np.float32)
    # adjacent equal peaks
    a[5, 5] = a[5, 6] = 2.0
    a[10, 10] = a[11, 10] = 2.0
    # flat plateau
    a[14:17, 3:6] = 3.0
    # border ties (inner-map border rows/cols 0 and -1 -> map rows 1, -2)
    a[1, 12] = 2.5
    a[2, 12] = 2.5
    a[1, 20] = 1.7
    a[3, 20] = 1.7  # reflected copy at r=... tie with reflection
    a[18, 1] = 1.9
    a[18, 3] = 1.9
    maps.append(a)
    b = np.full((20, 28), 0.95, np.float32)   # fully flat map (no peaks -> n=128 fill)
    b[6, 7] = 1.5
    maps.append(b)
    c = (rs.randint(0, 4, (20, 28)).astype(np.float32) / 3.0).astype(np.float32)  # many exact ties
    maps.append(c)
    d = rs.randn(20, 28).astype(np.float32)   # negative values
    maps.append(d)
    return [m[None, None] for m in maps]


sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_cfg import DET_CONFIGS, CRAFTED_CONFIGS  # noqa: E402


def gen_detector(out):
    res = {}
    for s in range(3):
        km = torch.from_numpy(np.random.RandomState(s).rand(1, 1, 480, 640).astype(np.float32))
        for name, r, n, un, thr, tm in DET_CONFIGS:
            d = ref_detect_with_idx(km, r, n, un, thr, tm)
            for k, v in d.items():
                res["rand%d_%s_%s" % (s, name, k)] = v
    for j, m in enumerate(crafted_maps()):
        km = torch.from_numpy(m)
        res["crafted%d_map" % j] = m
        for name, r, n, un, thr, tm in CRAFTED_CONFIGS:
            d = ref_detect_with_idx(km, r, n, un, thr, tm)
            for k, v in d.items():
                res["crafted%d_%s_%s" % (j, name, k)] = v
    np.savez_compressed(out, **res)


@torch.no_grad()
def gen_sampler(out):
    rs = np.random.RandomState(11)
    fmap = rs.randn(2, 128, 24, 32).astype(np.float32)
    coords = rs.uniform(-1.1, 1.1, (2, 160, 2)).astype(np.float32)
    coords[:, :4] = [[-1, -1], [1, 1], [-1, 1], [0, 0]]
    t_f, t_c = torch.from_numpy(fmap), torch.from_numpy(coords)
    res = {"coords": coords,
           "desc_norm": ref_putils.sample_feat_by_coord(t_f, t_c, True).numpy(),
           "desc_raw": ref_putils.sample_feat_by_coord(t_f, t_c, False).numpy(),
           "denorm": ref_putils.denormalize_coords(t_c, 480, 640).numpy(),
           "renorm": ref_putils.normalize_coords(ref_putils.denormalize_coords(t_c, 480, 640),
                                                 480, 640).numpy()}
    np.savez_compressed(out, **res)


def gen_model_small(out):
    bb, hd = build_ref_models(0)
    res = {}
    for tag, (h, w, i) in {"a": (96, 128, 0), "b": (64, 96, 1)}.items():
        img = torch.from_numpy(seeded_image(i, h, w))[None]
        o = ref_extract(bb, hd, img)
        for k, v in o.items():
            res["%s_%s" % (tag, k)] = v.numpy()
        d = ref_detect_with_idx(o["local_point"], 1, 256, True, 0.9, "abs")
        for k, v in d.items():
            res["%s_det_%s" % (tag, k)] = v
        cn = torch.from_numpy(d["coord_n"])
        res["%s_desc" % tag] = ref_putils.sample_feat_by_coord(o["local_map"], cn, True).numpy()
    np.savez_compressed(out, **res)


def gen_extract_full(out):
    bb, hd = build_ref_models(0)
    img = torch.from_numpy(seeded_image(0, 480, 640))[None]
    o = ref_extract(bb, hd, img)
    lp = o["local_point"]
    d = ref_detect_with_idx(lp, 1, 2048, True, 0.9, "abs")
    cn = torch.from_numpy(d["coord_n"])
    desc = ref_putils.sample_feat_by_coord(o["local_map"], cn, True).numpy()
    kpt = ref_putils.denormalize_coords(cn, 480, 640).numpy()
    res = {"idx": d["idx"], "coord_n": d["coord_n"], "kp_score": d["kp_score"],
           "count": d["count"], "masked": d["masked"], "kpt": kpt,
           "desc_first256": desc[:, :256],
           "local_point_rows": lp[0, 0, ::40].numpy(),          # 12 full rows
           "local_map_px": o["local_map"][0, :, ::20, ::20].numpy(),  # 6x8 pixels
           "global_feat": o["global_feat"].numpy(),
           "local_point_sum": np.float64(lp.double().sum()),
           "local_map_sum": np.float64(o["local_map"].double().sum()),
           "global_map_sum": np.float64(o["global_map"].double().sum())}
    np.savez_compressed(out, **res)


def synthetic_fundamental(b, h, w, seed):
    """F1/F2 from K, R, t exactly as datasets/megadepth.py:426-448 builds them
    (E = [t]x R, F = K2^-T E K1^-1, normalised by F[2,2]); K with f = w*0.8,
    principal point at the centre, R = exp(small rotvec), t = random unit."""
    from posfeat_amd.correlation import synthetic_fundamental as sf
    return sf(b, h, w, seed)


DESC_CFG = {"kps_generator": "generate_kpts_regular_grid_random",
            "kps_generator_config": {"grid_size": 16, "map_init": "identity",
                                     "keep_spatial": True, "random_select": "random"},
            "window_size": 0.1, "loss_distance": "cos", "use_nn_grid": False,
            "use_line_search": True,
            "line_search_config": {"line_step": 100, "use_nn": True, "loc_rand": True},
            "temperature_base": 60, "temperature_max": 60}
EPI_CFG = {"grid_cost_thr": 0.5, "win_cost_thr": 0.1, "use_std_as_weight": True,
           "weight_grid": 0, "weight_window": 1}
DISK_CFG = {"grid_size": 8, "loss_distance": "cos", "temperature_base": 60,
            "temperature_max": 60, "epipolar_reward": "constant_reward",
            "reward_config": {"reward_thr": 2, "rescale_thr": False}, "cor_detach": True,
            "good_reward": 1, "bad_reward": -0.25, "kp_penalty": -0.001, "match_grad": False}


def corr_inputs(b, H, W, seed):
    rs = np.random.RandomState(seed)
    xf1 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    xf2 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    # smooth the maps a little so correlations have structure
    xf1 = F.avg_pool2d(xf1, 3, 1, 1)
    xf2 = F.avg_pool2d(xf2, 3, 1, 1)
    kp1 = torch.from_numpy(rs.rand(b, 1, H, W).astype(np.float32) * 3)
    kp2 = torch.from_numpy(rs.rand(b, 1, H, W).astype(np.float32) * 3)
    F1, F2 = synthetic_fundamental(b, H, W, seed)
    return xf1, xf2, kp1, kp2, torch.from_numpy(F1), torch.from_numpy(F2)


@torch.no_grad()
def gen_correlation(out):
    res = {}
    for tag, (b, H, W, seed) in {"s": (2, 240, 320, 3), "f": (1, 480, 640, 4)}.items():
        xf1, xf2, kp1, kp2, F1, F2 = corr_inputs(b, H, W, seed)
        inputs = {"im1": torch.zeros(b, 3, H, W), "im2": torch.zeros(b, 3, H, W), "F1": F1, "F2": F2}
        outputs = {"preds1": {"global_map": xf1[:, :, ::4, ::4], "local_map": xf1,
                              "local_point": kp1},
                   "preds2": {"global_map": xf2[:, :, ::4, ::4], "local_map": xf2,
                              "local_point": kp2}, "epoch": 0}
        pre = ref_losses.Preprocess_Line2Window(DESC_CFG)
        torch.manual_seed(100 + seed)
        proc = pre(inputs, outputs)
        # replay the RNG draws (same seed, same call sequence)
        torch.manual_seed(100 + seed)
        k1, k2, _, _ = ref_putils.generate_kpts_regular_grid_random(
            inputs, outputs, **DESC_CFG["kps_generator_config"])
        n = k1.shape[1] * k1.shape[2]
        r1 = torch.rand(b, n, 2)
        r2 = torch.rand(b, n, 2)
        for name, k, hh, ww in (("sel1", k1, H, W), ("sel2", k2, H, W)):
            ix = torch.round((k[..., 0] + 1) / 2 * (ww - 1)).long()
            iy = torch.round((k[..., 1] + 1) / 2 * (hh - 1)).long()
            res["%s_%s" % (tag, name)] = ((iy % 16) * 16 + ix % 16).int().numpy()
        res[tag + "_rand1"] = r1.numpy()
        res[tag + "_rand2"] = r2.numpy()
        for k, v in proc.items():
            if torch.is_tensor(v):
                res["%s_proc_%s" % (tag, k)] = v.numpy()
        loss, comp = ref_losses.EpipolarLoss_full(EPI_CFG)(inputs, outputs, proc)
        res[tag + "_epi_loss"] = loss.numpy()
        for k, v in comp.items():
            res["%s_epi_%s" % (tag, k)] = v.numpy()
        # DiskLoss on the same maps
        dl = ref_losses.DiskLoss(DISK_CFG)
        torch.manual_seed(200 + seed)
        dloss, dcomp = dl(inputs, outputs, None)
        torch.manual_seed(200 + seed)
        for i, km in ((1, kp1), (2, kp2)):
            kps, logp, acc = dl.point_sample(km)
            ix, iy = kps[..., 0].long(), kps[..., 1].long()
            res["%s_prop%d" % (tag, i)] = ((iy % 8) * 8 + ix % 8).int().numpy()[:, None]
            res["%s_acc%d" % (tag, i)] = acc.numpy()
        res[tag + "_disk_loss"] = dloss.numpy()
        for k in ("reinforce", "kp_penalty", "n_kps"):
            res["%s_disk_%s" % (tag, k)] = dcomp[k].numpy()
    np.savez_compressed(out, **res)


DESC_GRAD_CASES = {"m": (1, 160, 224, 7), "l": (1, 240, 320, 8)}


def gen_desc_grad(out):
    """Descriptor-training loss gradient on the reference's own modules:
    Preprocess_Line2Window + EpipolarLoss_full (train_desc.yaml configs) with
    the local maps as autograd leaves, loss.backward() (trainer.py:331).
    Case m: full dL/d maps; case l: every 4th pixel in each direction plus
    full-map sums.  Draws replayed as in gen_correlation."""
    res = {}
    for tag, (b, H, W, seed) in DESC_GRAD_CASES.items():
        xf1, xf2, _, _, F1, F2 = corr_inputs(b, H, W, seed)
        xf1.requires_grad_(True)
        xf2.requires_grad_(True)
        inputs = {"im1": torch.zeros(b, 3, H, W), "im2": torch.zeros(b, 3, H, W), "F1": F1, "F2": F2}
        kz = torch.zeros(b, 1, H, W)
        outputs = {"preds1": {"global_map": xf1[:, :, ::4, ::4], "local_map": xf1,
                              "local_point": kz},
                   "preds2": {"global_map": xf2[:, :, ::4, ::4], "local_map": xf2,
                              "local_point": kz}, "epoch": 0}
        pre = ref_losses.Preprocess_Line2Window(DESC_CFG)
        torch.manual_seed(100 + seed)
        proc = pre(inputs, outputs)
        loss, _ = ref_losses.EpipolarLoss_full(EPI_CFG)(inputs, outputs, proc)
        loss.backward()
        g1, g2 = xf1.grad.numpy(), xf2.grad.numpy()
        torch.manual_seed(100 + seed)
        k1, k2, _, _ = ref_putils.generate_kpts_regular_grid_random(
            inputs, outputs, **DESC_CFG["kps_generator_config"])
        n = k1.shape[1] * k1.shape[2]
        r1 = torch.rand(b, n, 2)
        r2 = torch.rand(b, n, 2)
        for name, k in (("sel1", k1), ("sel2", k2)):
            ix = torch.round((k[..., 0] + 1) / 2 * (W - 1)).long()
            iy = torch.round((k[..., 1] + 1) / 2 * (H - 1)).long()
            res["%s_%s" % (tag, name)] = ((iy % 16) * 16 + ix % 16).int().numpy()
        res[tag + "_rand1"] = r1.numpy()
        res[tag + "_rand2"] = r2.numpy()
        res[tag + "_loss"] = loss.detach().numpy()
        res[tag + "_w1"] = proc["feat1w_corloc"].detach().numpy()
        if tag == "m":
            res[tag + "_dxf1"], res[tag + "_dxf2"] = g1, g2
        else:
            res[tag + "_dxf1_sub"], res[tag + "_dxf2_sub"] = g1[:, :, ::4, ::4], g2[:, :, ::4, ::4]
            res[tag + "_dxf_sums"] = np.array([g1.astype(np.float64).sum(), np.abs(g1).sum(),
                                               g2.astype(np.float64).sum(), np.abs(g2).sum()])
    np.savez_compressed(out, **res)


TRAIN_KP_CASES ={"a": (2, 64, 96, 5, 300), "b": (1, 96, 128, 6, 301)}


def gen_train_kp(out):
    """Config-5 step on the reference's own modules: KeypointDet (DeteNet.py)
    in train mode on detached backbone maps (PoSFeat_model.py:97-102), the
    reference DiskLoss (kploss.py) with torch.manual_seed, loss.backward()
    through autograd (trainer.py:330-331).  Stores the loss, every head
    parameter's gradient and the replayed draws (same seed, same call order:
    point_sample(kp1) then point_sample(kp2), kploss.py:141-142)."""
    bb, hd = build_ref_models(0)
    res = {}
    for tag, (b, H, W, fseed, tseed) in TRAIN_KP_CASES.items():
        im1 = torch.from_numpy(np.stack([seeded_image(10 + i + 7 * fseed, H, W) for i in range(b)]))
        im2 = torch.from_numpy(np.stack([seeded_image(20 + i + 7 * fseed, H, W) for i in range(b)]))
        F1, F2 = synthetic_fundamental(b, H, W, fseed)
        F1, F2 = torch.from_numpy(F1), torch.from_numpy(F2)
        hd.train()
        hd.zero_grad()
        preds = {}
        for key, im in (("preds1", im1), ("preds2", im2)):
            with torch.no_grad():
                feat = bb(im)
            local_input = torch.cat([feat["local_map"], feat["local_map_small"]], dim=1).detach()
            lp = hd([local_input, im])
            preds[key] = {"local_map": feat["local_map"], "local_point": lp,
                          "global_map": feat["global_map"]}
        outputs = dict(preds, epoch=1)
        inputs = {"im1": im1, "im2": im2, "F1": F1, "F2": F2}
        dl = ref_losses.DiskLoss(DISK_CFG)
        torch.manual_seed(tseed)
        loss, comp = dl(inputs, outputs, None)
        loss.backward()
        res[tag + "_loss"] = loss.detach().numpy()
        for k in ("reinforce", "kp_penalty", "n_kps"):
            res["%s_%s" % (tag, k)] = comp[k].detach().numpy()
        for k, p in hd.named_parameters():
            res["%s_grad_%s" % (tag, k)] = p.grad.detach().numpy().copy()
        torch.manual_seed(tseed)
        for i, key in ((1, "preds1"), (2, "preds2")):
            kps, _, acc = dl.point_sample(preds[key]["local_point"].detach())
            ix, iy = kps[..., 0].long(), kps[..., 1].long()
            res["%s_prop%d" % (tag, i)] = ((iy % 8) * 8 + ix % 8).int().numpy()[:, None]
            res["%s_acc%d" % (tag, i)] = acc.numpy()
            res["%s_lp%d" % (tag, i)] = preds[key]["local_point"].detach().numpy()
        hd.eval()
    np.savez_compressed(out, **res)


BB_GRAD_CASE = (2, 128, 160, 9)


def gen_bb_grad(out):
    """Config-3 backbone step on the reference's own ResUNet (DescNet.py) in
    train mode (trainer.py:293-296): two backbone calls (im1, im2:
    PoSFeat_model.py:144-145 -- separate BatchNorm batch statistics, running
    statistics updated twice), loss = sum(local_map1 * R1) + sum(local_map2 *
    R2) with seeded cotangents R (any dL/d local_map drives the same
    backward), loss.backward().  Stores the local maps (every 2nd pixel), per
    parameter [sum g, sum |g|, sum g^2] (fp64), full gradients of tensors of
    <= 40000 elements, 512 seeded entries of the larger ones, and the running
    statistics after both forwards.  conv_coarse gets no gradient (global_map
    is not in the loss)."""
    import zlib
    bb, _ = build_ref_models(0)
    b, H, W, seed = BB_GRAD_CASE
    im1 = torch.from_numpy(np.stack([seeded_image(30 + i, H, W) for i in range(b)]))
    im2 = torch.from_numpy(np.stack([seeded_image(40 + i, H, W) for i in range(b)]))
    rs = np.random.RandomState(seed)
    R1 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    R2 = torch.from_numpy(rs.randn(b, 128, H // 4, W // 4).astype(np.float32))
    bb.train()
    bb.zero_grad()
    o1 = bb(im1)
    o2 = bb(im2)
    loss = (o1["local_map"] * R1).sum() + (o2["local_map"] * R2).sum()
    loss.backward()
    res = {"lm1_sub": o1["local_map"].detach()[:, :, ::2, ::2].numpy().copy(),
           "lm2_sub": o2["local_map"].detach()[:, :, ::2, ::2].numpy().copy(),
           "loss": loss.detach().numpy()}
    for k, p in bb.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().numpy()
        g64 = g.astype(np.float64)
        res["stat_" + k] = np.array([g64.sum(), np.abs(g64).sum(), (g64 * g64).sum()])
        if g.size <= 40000:
            res["grad_" + k] = g.copy()
        else:
            idx = np.random.RandomState(zlib.crc32(k.encode())).choice(g.size, 512, replace=False)
            res["idx_" + k] = idx.astype(np.int64)
            res["val_" + k] = g.reshape(-1)[idx].copy()
    for k, v in bb.state_dict().items():
        if "running" in k:
            res["rs_" + k] = v.numpy().copy()
    bb.eval()
    # the same step on the reference modules in fp64: the fp32 gradients of this
    # 13-block train-mode network carry up to ~3e-2 relative rounding noise
    # (BatchNorm backward cancels), so the HIP path is judged against fp64 with
    # a per-tensor tolerance set by the reference's own fp32 error ("noise_")
    bb64, _ = build_ref_models(0)
    bb64 = bb64.double()
    bb64.train()
    bb64.zero_grad()
    p1 = bb64(im1.double())
    p2 = bb64(im2.double())
    ((p1["local_map"] * R1.double()).sum() + (p2["local_map"] * R2.double()).sum()).backward()
    for k, p in bb64.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().numpy()
        if "grad_" + k in res:
            res["g64_" + k] = g.copy()
            ref32 = res["grad_" + k].astype(np.float64)
            g = g.reshape(ref32.shape)
        else:
            g = g.reshape(-1)[res["idx_" + k]]
            res["v64_" + k] = g.copy()
            ref32 = res["val_" + k].astype(np.float64)
        res["noise_" + k] = np.array(np.abs(ref32 - g).max() / max(np.abs(g).max(), 1e-300))
    np.savez_compressed(out, **res)


# evaluation matchers: the reference's own functions on seeded
# descriptor sets (oracle.match_ref.seeded_descriptors regenerates the inputs)
MATCH_CASES = [(11, 1000, 1200), (12, 2048, 2048), (13, 500, 300), (14, 4096, 3000)]


def gen_matchers(out):
    from oracle.match_ref import seeded_descriptors
    am = _load("ref_aachen_matchers", os.path.join(REF, "evaluations", "aachen", "matchers.py"))
    em = _load("ref_eth_matchers", os.path.join(REF, "evaluations", "ETH_local_feature",
                                                 "custom_matcher.py"))
    res = {}
    for seed, n1, n2 in MATCH_CASES:
        d1, d2 = seeded_descriptors(seed, n1, n2)
        t1, t2 = torch.from_numpy(d1), torch.from_numpy(d2)
        tag = "m%d" % seed
        res[tag + "_shape"] = np.array([n1, n2], np.int64)
        res[tag + "_mnn"] = ref_putils.mnn_matcher(t1, t2)
        res[tag + "_mutual_nn"] = am.mutual_nn_matcher(t1, t2)
        res[tag + "_eth_mutual_nn"] = em.mutual_nn_matcher(t1, t2)
        for r in (0.95, 0.8):
            res["%s_ratio_%g" % (tag, r)] = am.ratio_matcher(t1, t2, ratio=r)
            res["%s_mnn_ratio_%g" % (tag, r)] = am.mutual_nn_ratio_matcher(t1, t2, ratio=r)
    np.savez_compressed(out, **res)


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    which = sys.argv[1:] or ["detector", "sampler", "model_small", "extract_full", "correlation",
                             "train_kp"]
    if "train_kp" in which:
        gen_train_kp(os.path.join(HERE, "train_kp.npz"))
    if "desc_grad" in which:
        gen_desc_grad(os.path.join(HERE, "desc_grad.npz"))
    if "bb_grad" in which:
        gen_bb_grad(os.path.join(HERE, "bb_grad.npz"))
    if "detector" in which:
        gen_detector(os.path.join(HERE, "detector.npz"))
    if "sampler" in which:
        gen_sampler(os.path.join(HERE, "sampler.npz"))
    if "model_small" in which:
        gen_model_small(os.path.join(HERE, "model_small.npz"))
    if "extract_full" in which:
        gen_extract_full(os.path.join(HERE, "extract_full.npz"))
    if "correlation" in which:
        gen_correlation(os.path.join(HERE, "correlation.npz"))
    if "matchers" in which:
        gen_matchers(os.path.join(HERE, "matchers.npz"))
    print("golden fixtures written to", HERE)
