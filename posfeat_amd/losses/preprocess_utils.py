"""Drop-in for the hot-path functions of losses/preprocess_utils.py.

Same names, arguments and return shapes as the reference; GPU tensors go
through the HIP kernels of libposfeat_hip.so.  Options the reference's
configs never select (stable=False gumbel sampling, 'softnms') raise
NotImplementedError rather than fall back.

  normalize_coords      preprocess_utils.py:14-26
  denormalize_coords    preprocess_utils.py:28-38
  sample_feat_by_coord  preprocess_utils.py:40-53
  gen_grid              preprocess_utils.py:84-87
  generate_kpts_single  preprocess_utils.py:215-278
  nms                   preprocess_utils.py:449-464
  mnn_matcher           preprocess_utils.py:795-803
"""
import torch

from .. import ops


def homogenize(coord):
    return torch.cat((coord, torch.ones_like(coord[..., [0]])), -1)


def normalize_coords(coord, h, w):
    c = torch.tensor([(w - 1) / 2.0, (h - 1) / 2.0], dtype=torch.float32, device=coord.device)
    return (coord - c) / c


def denormalize_coords(coord_norm, h, w):
    c = torch.tensor([(w - 1) / 2.0, (h - 1) / 2.0], dtype=torch.float32,
                     device=coord_norm.device)
    return coord_norm * c + c


def gen_grid(h_min, h_max, w_min, w_max, len_h, len_w):
    x = torch.linspace(w_min, w_max, len_w)
    y = torch.linspace(h_min, h_max, len_h)
    yy, xx = torch.meshgrid(y, x, indexing="ij")
    return torch.stack((xx, yy), -1).reshape(-1, 2).float()


def sample_feat_by_coord(x, coord_n, norm=False, nhwc=None):
    """x: [b,c,h,w] feature map, coord_n: [b,n,2] -> [b,n,c].

    ``nhwc`` (optional) is an NHWC copy of ``x`` (e.g. the engine's
    ``ExtractOutputs.local_map_nhwc``); without it the map is relaid out once
    by the HIP layout kernel."""
    b, c, h, w = x.shape
    if nhwc is None:
        nhwc = ops.nchw_to_nhwc(x.float().contiguous())
    return ops.sample_desc_nhwc(nhwc, coord_n.float(), c=c, normalize=bool(norm))


def generate_kpts_single(kp_map, nms_radius, num_pts=False, scale=4, stable=True, temperature=1,
                         stride=1, use_nms=True, thr=False, thr_mod="mean"):
    _, coord, score, _, _ = _detect(kp_map, nms_radius, num_pts, stable, stride, use_nms, thr,
                                    thr_mod, sync=True)
    return coord, score


def generate_kpts_single_async(kp_map, nms_radius, num_pts=False, scale=4, stable=True,
                               temperature=1, stride=1, use_nms=True, thr=False, thr_mod="mean"):
    """generate_kpts_single without the host synchronisation: full-capacity
    (coord_n [b,cap,2], kp_score [b,cap,1]) plus the number of selected
    keypoints n as a one-element device tensor (rows beyond n are unused).
    n is the reference's (preprocess_utils.py:249-261): min(num_pts, the
    smallest survivor count of the batch), raised to 128 -- NOT the survivor
    count itself, which is smaller than n whenever the raise pads top-k with
    zero-score entries (a 128 x 160 Aachen image at r = 3 has ~75 survivors)."""
    _, coord, score, _, n_sel = _detect(kp_map, nms_radius, num_pts, stable, stride, use_nms,
                                        thr, thr_mod, sync=False)
    return coord, score, n_sel


def generate_kpts_each_async(kp_map, nms_radius, num_pts=False, scale=4, stable=True,
                             temperature=1, stride=1, use_nms=True, thr=False, thr_mod="mean"):
    """generate_kpts_single_async for a batch of same-size images, each
    selected as if it were detected alone (the reference extractor calls
    generate_kpts_single per image, batch_size 1): n is a device tensor [b]."""
    if not stable:
        raise NotImplementedError("stable=False (gumbel sampling) is not implemented")
    if use_nms == "softnms":
        raise NotImplementedError("use_nms='softnms' is not implemented")
    if stride != 1:
        raise NotImplementedError("stride != 1 is not implemented")
    _, coord, score, _, n_sel = ops.detect(kp_map.float().contiguous(), nms_radius, num_pts,
                                           use_nms=bool(use_nms), thr=thr, thr_mod=thr_mod,
                                           sync=False, each=True)
    return coord, score, n_sel


def _detect(kp_map, nms_radius, num_pts, stable, stride, use_nms, thr, thr_mod, sync):
    if not stable:
        raise NotImplementedError("stable=False (gumbel sampling) is not implemented")
    if use_nms == "softnms":
        raise NotImplementedError("use_nms='softnms' is not implemented")
    if stride != 1:
        raise NotImplementedError("stride != 1 is not implemented")
    return ops.detect(kp_map.float().contiguous(), nms_radius, num_pts, use_nms=bool(use_nms),
                      thr=thr, thr_mod=thr_mod, sync=sync)


def nms(score, patch_radius):
    """Bool mask of window maxima of ``score`` [b,1,h,w] (reflect padding,
    first-occurrence tie rule; preprocess_utils.py:449-464)."""
    return ops.nms_mask(score.float().contiguous(), patch_radius)


def mnn_matcher(descriptors_a, descriptors_b):
    """Mutual nearest neighbours (preprocess_utils.py:795-803) on the fused
    MFMA similarity + arg-max kernel (posfeat_amd.matchers)."""
    from ..matchers import mnn_matcher as _mnn
    return _mnn(descriptors_a, descriptors_b)
