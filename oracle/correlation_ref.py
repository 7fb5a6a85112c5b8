"""torch-CPU fp32 restatement of the training-side descriptor correlation
(TEST ORACLE).  Random draws are explicit inputs so the same values can be
fed to the HIP kernels:

* ``grid_points``            generate_kpts_regular_grid_random(_single),
                             preprocess_utils.py:598-659 (identity map,
                             random_select='random', keep_spatial=True);
                             ``sel`` = the Categorical sample per 16x16 cell
* ``line2window``            Preprocess_Line2Window.forward, preprocess.py:27-121
  - ``epipolar_line_search`` preprocess_utils.py:661-694 (``rand`` = the
                             torch.rand draw of loc_rand)
  - ``get_endpoints``        preprocess_utils.py:696-719
  - ``window_expectation``   get_expected_correspondence_within_window, 721-758
* ``epipolar_loss``          EpipolarLoss_full.forward, epipolarloss.py:38-101
* ``disk_loss``              DiskLoss.forward with constant_reward,
                             kploss.py:20-89, 132-197 (``proposals`` and
                             ``accept`` = the Categorical / Bernoulli draws)
"""
import torch
import torch.nn.functional as F


def gen_grid(h_min, h_max, w_min, w_max, len_h, len_w):
    y, x = torch.meshgrid(torch.linspace(h_min, h_max, len_h), torch.linspace(w_min, w_max, len_w),
                          indexing="ij")
    return torch.stack((x, y), -1).reshape(-1, 2).float()


def normalize_coords(coord, h, w):
    c = torch.tensor([(w - 1) / 2.0, (h - 1) / 2.0], dtype=torch.float32)
    return (coord - c) / c


def denormalize_coords(coord_n, h, w):
    c = torch.tensor([(w - 1) / 2.0, (h - 1) / 2.0], dtype=torch.float32)
    return coord_n * c + c


def homogenize(coord):
    return torch.cat((coord, torch.ones_like(coord[..., [0]])), -1)


def sample_feat(x, coord_n, norm):
    f = F.grid_sample(x, coord_n.unsqueeze(2), padding_mode="zeros", align_corners=False).squeeze(-1)
    if norm:
        f = F.normalize(f, p=2, dim=1)
    return f.transpose(1, 2)


def grid_points(sel, h, w, g):
    """sel: [b, h//g, w//g] int in [0, g*g) -> normalised coords [b, (h//g)*(w//g), 2]."""
    b, hc, wc = sel.shape
    xs = torch.linspace(-1, 1, w)
    ys = torch.linspace(-1, 1, h)
    ry, rx = sel // g, sel % g
    iy = torch.arange(hc).view(1, hc, 1) * g + ry
    ix = torch.arange(wc).view(1, 1, wc) * g + rx
    return torch.stack([xs[ix], ys[iy]], -1).reshape(b, -1, 2)


def get_endpoints(coords, Fmat, h, w):
    b, n, _ = coords.shape
    line = Fmat.bmm(homogenize(coords).transpose(1, 2))
    a, bb, c = line[:, 0, :], line[:, 1, :], line[:, 2, :]
    pl = torch.stack([torch.zeros_like(a), -c / bb], -1)
    pr = torch.stack([(w - 1) * torch.ones_like(a), -(a * (w - 1) + c) / bb], -1)
    pu = torch.stack([-(bb * (h - 1) + c) / a, (h - 1) * torch.ones_like(a)], -1)
    pb = torch.stack([-c / a, torch.zeros_like(a)], -1)
    pts = torch.stack([pl, pr, pu, pb], -1).transpose(2, 3)
    mask = (pts[:, :, :, 0] >= 0) & (pts[:, :, :, 0] <= w - 1) & (pts[:, :, :, 1] >= 0) & \
        (pts[:, :, :, 1] <= h - 1)
    valid = mask.sum(-1) == 2
    mask[~valid] = torch.tensor([True, True, False, False])
    pts = pts[mask].reshape(b, n, 2, 2)
    return normalize_coords(pts[:, :, 0], h, w), normalize_coords(pts[:, :, 1], h, w), valid


def epipolar_line_search(coord, Fmat, feat1, featmap2, h, w, rand, line_step=100,
                         window_size=0.1):
    b, n = coord.shape[:2]
    d = featmap2.shape[1]
    e1, e2, valid = get_endpoints(coord, Fmat, h, w)
    t = torch.stack([torch.linspace(0.0, 1.0, line_step)] * 2, -1)
    grids = (e2 - e1)[:, :, None, :] * t[None, None] + e1[:, :, None, :]
    pts = F.grid_sample(featmap2, grids, padding_mode="border", align_corners=False).permute(0, 2, 3, 1)
    sim = feat1.reshape(b * n, 1, d).bmm(pts.reshape(b * n, line_step, d).transpose(1, 2))
    prob = F.softmax(sim, dim=-1).reshape(b, n, line_step)
    mask = prob == prob.max(-1, True)[0]
    exp_org = (mask.unsqueeze(-1) * grids).sum(2)
    expected = exp_org + 0.707 * window_size * (2 * rand - 1)
    border = (expected[:, :, 0] >= -1) & (expected[:, :, 0] <= 1) & (expected[:, :, 1] >= -1) & \
        (expected[:, :, 1] <= 1)
    valid = valid & border
    var = (grids ** 2 * prob.unsqueeze(-1)).sum(2) - expected ** 2
    std = torch.sqrt(torch.clamp(var, min=1e-10)).sum(-1)
    return expected, exp_org, valid, std


def window_expectation(feat1, featmap2, center_n, window_size):
    b, d, h2, w2 = featmap2.shape
    n = center_n.shape[1]
    grid_n = gen_grid(-window_size, window_size, -window_size, window_size,
                      int(window_size * h2), int(window_size * w2))
    g = center_n.unsqueeze(-2) + grid_n.view(1, 1, -1, 2)
    win = F.grid_sample(featmap2, g, padding_mode="zeros", align_corners=False).permute(0, 2, 3, 1)
    sim = feat1.reshape(b * n, 1, d).bmm(win.reshape(b * n, -1, d).transpose(1, 2))
    prob = F.softmax(sim, dim=-1).reshape(b, n, -1)
    expected = (g * prob.unsqueeze(-1)).sum(2)
    var = (g ** 2 * prob.unsqueeze(-1)).sum(2) - expected ** 2
    std = torch.sqrt(torch.clamp(var, min=1e-10)).sum(-1)
    return expected, g, std


@torch.no_grad()
def line2window(xf1, xf2, F1, F2, im_hw1, im_hw2, sel1, sel2, rand1, rand2, temperature=60.0,
                grid_size=16, window_size=0.1, line_step=100):
    """Preprocess_Line2Window.forward for the train_desc.yaml configuration."""
    h1i, w1i = im_hw1
    h2i, w2i = im_hw2
    b = xf1.shape[0]
    c1n = grid_points(sel1, h1i, w1i, grid_size)
    c2n = grid_points(sel2, h2i, w2i, grid_size)
    coord1 = denormalize_coords(c1n, h1i, w1i)
    coord2 = denormalize_coords(c2n, h2i, w2i)
    f1 = sample_feat(xf1, c1n, True)
    f2 = sample_feat(xf2, c2n, True)
    cos = f1 @ f2.transpose(1, 2)
    p_row = F.softmax(temperature * cos, dim=2)
    p_col = F.softmax(temperature * cos, dim=1)
    g1 = (p_row.unsqueeze(-1) * coord2.unsqueeze(1)).sum(2)
    g2 = (p_col.unsqueeze(-1) * coord1.unsqueeze(2)).sum(1)
    g1n = normalize_coords(g1, h2i, w2i)
    g2n = normalize_coords(g2, h1i, w1i)
    s1 = (p_row.unsqueeze(-1) * (c2n.reshape(b, 1, -1, 2) ** 2)).sum(2) - g1n ** 2
    s1 = s1.clamp(min=1e-6).sqrt().sum(-1)
    s2 = (p_col.unsqueeze(-1) * (c1n.reshape(b, -1, 1, 2) ** 2)).sum(1) - g2n ** 2
    s2 = s2.clamp(min=1e-6).sqrt().sum(-1)
    fm2 = temperature * F.normalize(xf2, p=2.0, dim=1)
    fm1 = temperature * F.normalize(xf1, p=2.0, dim=1)
    l1, l1_org, v1, _ = epipolar_line_search(coord1, F1, f1, fm2, h2i, w2i, rand1, line_step,
                                             window_size)
    l2, l2_org, v2, _ = epipolar_line_search(coord2, F2, f2, fm1, h1i, w1i, rand2, line_step,
                                             window_size)
    w1n, _, w1s = window_expectation(f1, fm2, l1, window_size)
    w2n, _, w2s = window_expectation(f2, fm1, l2, window_size)
    return {"coord1": coord1, "coord2": coord2, "feat1g_corloc": g1, "feat2g_corloc": g2,
            "feat1w_corloc": denormalize_coords(w1n, h2i, w2i),
            "feat2w_corloc": denormalize_coords(w2n, h1i, w1i),
            "feat1c_corloc_org": denormalize_coords(l1_org, h2i, w2i),
            "feat2c_corloc_org": l2_org,  # sic: the reference returns the normalised one
            "feat1g_std": s1, "feat2g_std": s2, "feat1w_std": w1s, "feat2w_std": w2s,
            "temperature": temperature, "valid_epi1": v1, "valid_epi2": v2}


def _epipolar_cost(c1, c2, Fm):
    line = Fm.bmm(homogenize(c1).transpose(1, 2))
    line = line / torch.clamp(torch.norm(line[:, :2, :], dim=1, keepdim=True), min=1e-8)
    return torch.abs(torch.sum(homogenize(c2).transpose(1, 2) * line, dim=1))


def _set_weight(inv_std, mask):
    w = inv_std / torch.mean(inv_std)
    w = w * mask.float()
    return w / (torch.mean(w) + 1e-8)


def epipolar_loss(processed, F1, F2, im_hw1, grid_cost_thr=0.5, win_cost_thr=0.1, w_g=0.0,
                  w_w=1.0):
    """EpipolarLoss_full.forward (use_std_as_weight=True)."""
    short = min(im_hw1)
    p = processed
    cg1 = _epipolar_cost(p["coord1"], p["feat1g_corloc"], F1)
    cw1 = _epipolar_cost(p["coord1"], p["feat1w_corloc"], F1)
    cg2 = _epipolar_cost(p["coord2"], p["feat2g_corloc"], F2)
    cw2 = _epipolar_cost(p["coord2"], p["feat2w_corloc"], F2)
    mg1 = (cg1 < short * grid_cost_thr) & p["valid_epi1"]
    mw1 = (cw1 < short * win_cost_thr) & p["valid_epi1"]
    mg2 = (cg2 < short * grid_cost_thr) & p["valid_epi2"]
    mw2 = (cw2 < short * win_cost_thr) & p["valid_epi2"]
    wg1 = _set_weight(1 / p["feat1g_std"].clamp(min=1e-10), mg1)
    ww1 = _set_weight(1 / p["feat1w_std"].clamp(min=1e-10), mw1)
    wg2 = _set_weight(1 / p["feat2g_std"].clamp(min=1e-10), mg2)
    ww2 = _set_weight(1 / p["feat2w_std"].clamp(min=1e-10), mw2)
    lg1, lw1 = (wg1 * cg1).mean(), (ww1 * cw1).mean()
    lg2, lw2 = (wg2 * cg2).mean(), (ww2 * cw2).mean()
    loss = w_g * (lg1 + lg2) + w_w * (lw1 + lw2)
    pg = (mg1.sum() / mg1.numel() + mg2.sum() / mg2.numel()) / 2
    pw = (mw1.sum() / mw1.numel() + mw2.sum() / mw2.numel()) / 2
    return loss, {"loss_g1": lg1, "loss_w1": lw1, "loss_g2": lg2, "loss_w2": lw2,
                  "percent_g": pg, "percent_w": pw}


def disk_point_logp(kp_map, g, proposals, accept):
    """logp of the per-cell Categorical proposal + Bernoulli acceptance and the
    chosen pixel coordinates (kploss.py:20-48)."""
    b, _, h, w = kp_map.shape
    un = kp_map.unfold(2, g, g).unfold(3, g, g).reshape(b, 1, h // g, w // g, g * g)
    lsm = torch.log_softmax(un, dim=-1)
    plogp = torch.gather(lsm, -1, proposals[..., None]).squeeze(-1)
    acc_logit = torch.gather(un, -1, proposals[..., None]).squeeze(-1)
    alogp = torch.where(accept, F.logsigmoid(acc_logit), F.logsigmoid(-acc_logit))
    ry, rx = proposals // g, proposals % g
    iy = torch.arange(h // g).view(1, 1, -1, 1) * g + ry
    ix = torch.arange(w // g).view(1, 1, 1, -1) * g + rx
    kps = torch.stack([ix.float(), iy.float()], -1).reshape(b, -1, 2)
    return kps, plogp + alogp


@torch.no_grad()
def disk_loss(kp1, kp2, xf1, xf2, F1, F2, prop1, prop2, acc1, acc2, temperature=60.0, g=8,
              reward_thr=2.0, good=1.0, bad=-0.25, kp_penalty=-0.001):
    """DiskLoss.forward value (constant_reward, rescale_thr False, cor_detach True)."""
    b, _, h, w = kp1.shape
    c1, logp1 = disk_point_logp(kp1, g, prop1, acc1)
    c2, logp2 = disk_point_logp(kp2, g, prop2, acc2)
    f1 = sample_feat(xf1, normalize_coords(c1, h, w), True)
    f2 = sample_feat(xf2, normalize_coords(c2, h, w), True)
    aff = -temperature * (1 - f1 @ f2.transpose(1, 2))
    lrow = torch.log_softmax(aff, dim=2)
    lcol = torch.log_softmax(aff, dim=1)
    dense_p = lrow.exp() * lcol.exp()
    dense_logp = lrow + lcol
    l1 = F1.bmm(homogenize(c1).transpose(1, 2))
    l1 = l1 / torch.clamp(torch.norm(l1[:, :2, :], p=2, dim=1, keepdim=True), min=1e-8)
    d1 = torch.abs(l1.transpose(1, 2) @ homogenize(c2).transpose(1, 2))
    l2 = F2.bmm(homogenize(c2).transpose(1, 2))
    l2 = l2 / torch.clamp(torch.norm(l2[:, :2, :], p=2, dim=1, keepdim=True), min=1e-8)
    d2 = torch.abs(l2.transpose(1, 2) @ homogenize(c1).transpose(1, 2)).transpose(1, 2)
    good_m = (d1 < reward_thr) & (d2 < reward_thr)
    reward = good * good_m + bad * (~good_m)
    kps_logp = logp1.reshape(b, 1, -1).transpose(1, 2) + logp2.reshape(b, 1, -1)
    plogp = dense_p * (dense_logp + kps_logp)
    am = acc1.reshape(b, 1, -1).transpose(1, 2) * acc2.reshape(b, 1, -1)
    reinforce = (reward[am] * plogp[am]).sum()
    penalty = kp_penalty * (logp1[acc1].sum() + logp2[acc2].sum())
    return -reinforce - penalty, {"reinforce": reinforce, "kp_penalty": penalty,
                                  "n_kps": (acc1.reshape(b, -1).sum(-1) +
                                            acc2.reshape(b, -1).sum(-1)).float().mean()}
