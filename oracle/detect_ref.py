"""numpy restatement of keypoint selection and descriptor sampling (TEST ORACLE).

Follows losses/preprocess_utils.py of the reference:

* ``gen_grid``            -- preprocess_utils.py:84-87
* ``normalize_coords``    -- preprocess_utils.py:14-26
* ``denormalize_coords``  -- preprocess_utils.py:28-38
* ``nms``                 -- preprocess_utils.py:449-464
* ``generate_kpts_single``-- preprocess_utils.py:215-278 (stable=True branch)
* ``sample_feat_by_coord``-- preprocess_utils.py:40-53

Tie rule, the one the HIP detector implements bit-exactly:

* NMS keeps pixel p iff S[p] is strictly greater than every element that
  precedes p's own position in the row-major scan of its reflect-padded
  (2r+1)^2 window and >= every element after it.  This is ATen's
  first-occurrence ``max_pool2d_with_indices`` followed by ``idx == coords``.
* top-k orders by (masked score descending, flat inner index ascending).
"""
import numpy as np


def gen_grid(h_min, h_max, w_min, w_max, len_h, len_w):
    """(len_h*len_w) x 2 grid of (x, y), row-major over (y, x)."""
    x = np.linspace(w_min, w_max, len_w).astype(np.float32)
    y = np.linspace(h_min, h_max, len_h).astype(np.float32)
    xx, yy = np.meshgrid(x, y)
    return np.stack([xx, yy], -1).reshape(-1, 2).astype(np.float32)


def normalize_coords(coord, h, w):
    c = np.array([(w - 1) / 2.0, (h - 1) / 2.0], np.float32)
    return ((coord - c) / c).astype(np.float32)


def denormalize_coords(coord_n, h, w):
    c = np.array([(w - 1) / 2.0, (h - 1) / 2.0], np.float32)
    return (coord_n * c + c).astype(np.float32)


def nms(score, r):
    """score: (h, w) float32 -> bool mask (h, w).  Reflect pad, first-occurrence argmax."""
    h, w = score.shape
    p = np.pad(score, r, mode="reflect")
    keep = np.ones((h, w), bool)
    center = r * (2 * r + 1) + r
    pos = 0
    for dy in range(2 * r + 1):
        for dx in range(2 * r + 1):
            if pos != center:
                sh = p[dy:dy + h, dx:dx + w]
                keep &= (sh < score) if pos < center else (sh <= score)
            pos += 1
    return keep


def _float_key(v):
    """Order-preserving uint32 key of float32 values (+0 == -0)."""
    v = (v.astype(np.float32) + np.float32(0.0)).view(np.uint32)
    return np.where(v & 0x80000000, ~v, v | 0x80000000).astype(np.uint32)


def topk_canonical(values, n):
    """Indices of the n largest values, ordered (value desc, index asc)."""
    key = _float_key(values).astype(np.int64)
    order = np.lexsort((np.arange(values.size), -key))
    return order[:n]


def detector_count(kp_map, nms_radius, use_nms=True, thr=False, thr_mod="mean"):
    """Number of surviving inner pixels per image (the reference's min-count input)."""
    _, mask = _mask_and_inner(kp_map, nms_radius, use_nms, thr, thr_mod)
    return mask.reshape(mask.shape[0], -1).sum(1)


def _mask_and_inner(kp_map, nms_radius, use_nms, thr, thr_mod):
    b, _, h, w = kp_map.shape
    inner = kp_map[:, 0, 1:-1, 1:-1]
    if use_nms:
        mask = np.stack([nms(inner[i], nms_radius) for i in range(b)])
    else:
        mask = np.ones(inner.shape, bool)
    if thr is not False and thr is not None and thr:
        if thr_mod == "max":
            kp_thr = inner.reshape(b, -1).max(1)
        elif thr_mod == "mean":
            kp_thr = inner.reshape(b, -1).astype(np.float32).mean(1, dtype=np.float32)
        else:  # 'abs'
            kp_thr = np.ones(b, np.float32)
        t = (np.float32(thr) * kp_thr.astype(np.float32)).astype(np.float32)
        mask &= inner > t[:, None, None]
    return inner, mask


def refine_maps(km):
    """Soft-argmax refinement of every inner pixel (preprocess_utils.py:243-246):
    avgpool3(kp * grid) / avgpool3(kp), normalised coordinates, for a (h, w)
    score map.  Returns (rx, ry), each (h-2, w-2) float32."""
    h, w = km.shape
    km = np.asarray(km, np.float64)
    grid = gen_grid(-1, 1, -1, 1, h, w).reshape(h, w, 2)
    gx = km * grid[..., 0]
    gy = km * grid[..., 1]

    def box(a):
        s = np.zeros((h - 2, w - 2), np.float64)
        for dy in range(3):
            for dx in range(3):
                s += a[dy:dy + h - 2, dx:dx + w - 2]
        return s / 9.0
    wgt = box(km)
    return (box(gx) / wgt).astype(np.float32), (box(gy) / wgt).astype(np.float32)


def generate_kpts_single(kp_map, nms_radius, num_pts=False, use_nms=True, thr=False,
                         thr_mod="mean", return_idx=False):
    """kp_map: (b,1,h,w) float32.  Returns coord_n (b,n,2), kp_score (b,n,1)[, idx (b,n)]."""
    kp_map = np.asarray(kp_map, np.float32)
    b, _, h, w = kp_map.shape
    inner, mask = _mask_and_inner(kp_map, nms_radius, use_nms, thr, thr_mod)
    counts = mask.reshape(b, -1).sum(1)
    if not num_pts:
        n = int(counts.min())
    else:
        n = int(num_pts)
        if n > counts.min():
            n = int(counts.min())
    if n < 128:
        n = 128
    coords, scores, idxs = [], [], []
    for i in range(b):
        rx, ry = refine_maps(kp_map[i, 0])
        mx = np.full((h - 2, w - 2), -np.inf, np.float32)
        for dy in range(3):
            for dx in range(3):
                mx = np.maximum(mx, kp_map[i, 0, dy:dy + h - 2, dx:dx + w - 2])
        masked = np.where(mask[i], inner[i], np.float32(0.0)).reshape(-1)
        idx = topk_canonical(masked, n)
        coords.append(np.stack([rx.reshape(-1)[idx], ry.reshape(-1)[idx]], -1))
        scores.append(mx.reshape(-1)[idx][:, None])
        idxs.append(idx)
    out = (np.stack(coords).astype(np.float32), np.stack(scores).astype(np.float32))
    if return_idx:
        out = out + (np.stack(idxs).astype(np.int64),)
    return out


def sample_feat_by_coord(x, coord_n, norm=False):
    """grid_sample(bilinear, zeros, align_corners=False) + optional L2 norm.

    x: (b,c,h,w), coord_n: (b,n,2) -> (b,n,c).  Computed in float64.
    """
    x = np.asarray(x, np.float64)
    b, c, h, w = x.shape
    out = np.zeros((b, coord_n.shape[1], c), np.float64)
    for i in range(b):
        gx = coord_n[i, :, 0].astype(np.float64)
        gy = coord_n[i, :, 1].astype(np.float64)
        ix = ((gx + 1) * w - 1) / 2
        iy = ((gy + 1) * h - 1) / 2
        x0 = np.floor(ix).astype(np.int64)
        y0 = np.floor(iy).astype(np.int64)
        for dy in (0, 1):
            for dx in (0, 1):
                xx = x0 + dx
                yy = y0 + dy
                wx = (ix - x0) if dx else (x0 + 1 - ix)
                wy = (iy - y0) if dy else (y0 + 1 - iy)
                ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
                v = np.zeros((coord_n.shape[1], c))
                v[ok] = x[i][:, yy[ok], xx[ok]].T
                out[i] += v * (wx * wy)[:, None]
    if norm:
        nrm = np.sqrt((out ** 2).sum(-1, keepdims=True))
        out = out / np.maximum(nrm, 1e-12)
    return out.astype(np.float32)


def process_image(local_point, local_map, detector_config, h, w):
    """Extractor.process for one image (managers/extractor.py:318-355, npz branch):
    detect -> denormalise with full-image h, w -> sample+L2 (loss_distance 'cos')."""
    cfg = dict(detector_config)
    coord_n, score, idx = generate_kpts_single(
        local_point, cfg.get("nms_radius", 1), cfg.get("num_pts", False),
        use_nms=cfg.get("use_nms", True), thr=cfg.get("thr", False),
        thr_mod=cfg.get("thr_mod", "mean"), return_idx=True)
    coords = denormalize_coords(coord_n, h, w)
    desc = sample_feat_by_coord(local_map, coord_n, True)
    return {"kpt": coords[0], "desc": desc, "kp_score": score, "idx": idx, "coord_n": coord_n}
