"""torch-tensor wrappers over the C ABI (device pointers + the current stream).

Every function here runs a hand-written gfx950 kernel; none has a CPU path.
Inputs must be contiguous fp32 CUDA(HIP) tensors on the current device.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr

ACT = {"none": 0, "relu": 1, "elu": 2}
THR_MODE = {"abs": 1, "max": 2, "mean": 3}


def _f32(t, name):
    if t.dtype != torch.float32:
        raise TypeError("%s must be float32 (got %s)" % (name, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    _lib.require_device(t)
    return t


def packed_k(cin, kh, kw):
    return lib().posfeat_conv_packed_k(cin, kh, kw)


def pack_conv_weight(w, b=None):
    """[Cout,Cin,KH,KW] (any device) -> (packed [Cout,Kpad] fp32, bias [Cout]) on w's device."""
    cout, cin, kh, kw = w.shape
    cinp = (cin + 3) // 4 * 4
    k = kh * kw * cinp
    kpad = packed_k(cin, kh, kw)
    out = torch.zeros(cout, kpad, dtype=torch.float32, device=w.device)
    if cin % 32 == 0:   # K = (cin/32, kh, kw, cin%32), see conv.hip
        wp = w.float().reshape(cout, cin // 32, 32, kh, kw).permute(0, 1, 3, 4, 2)
        out[:, :k] = wp.reshape(cout, k)
    else:               # K = (kh, kw, cin4), zero-padded
        wp = torch.zeros(cout, kh, kw, cinp, dtype=torch.float32, device=w.device)
        wp[..., :cin] = w.permute(0, 2, 3, 1).float()
        out[:, :k] = wp.reshape(cout, k)
    bias = b.float().contiguous() if b is not None else torch.zeros(cout, device=w.device)
    return out.contiguous(), bias


def conv2d_nhwc(x, w_packed, bias, cout, kh, kw, stride=1, pad=None, act="none", res=None,
                out=None, cin=None, allow_split=False):
    """Fused conv on an NHWC tensor x [n,h,w,cs] (first ``cin`` channels used).
    ``allow_split`` lets the library split K over workgroups (deterministic)."""
    _f32(x, "x")
    n, h, w, xcs = x.shape
    cin = xcs if cin is None else cin
    pad = (kh - 1) // 2 if pad is None else pad
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (w + 2 * pad - kw) // stride + 1
    if out is None:
        out = torch.empty(n, oh, ow, cout, device=x.device, dtype=torch.float32)
    d = _lib.ConvDesc(n=n, h=h, w=w, cin=cin, x_cstride=xcs, cout=cout, kh=kh, kw=kw,
                      stride=stride, pad=pad, y_cstride=out.shape[-1],
                      res_cstride=(res.shape[-1] if res is not None else 0), act=ACT[act])
    if allow_split:
        need = lib().posfeat_conv2d_workspace(ctypes.byref(d))
        ws = torch.empty(max(need, 16), dtype=torch.uint8, device=x.device)
        check(lib().posfeat_conv2d_nhwc_ws(ctypes.byref(d), ptr(x), ptr(_f32(w_packed, "w")),
                                           ptr(bias), ptr(res), ptr(out), ptr(ws), need,
                                           stream_ptr()))
        return out
    check(lib().posfeat_conv2d_nhwc(ctypes.byref(d), ptr(x), ptr(_f32(w_packed, "w")),
                                    ptr(bias), ptr(res), ptr(out), stream_ptr()))
    return out


def split_weight_planes(w_packed):
    """The packed [cout][Kpad] fp32 weights as three bf16 planes h, m, l
    (x = h + m + l up to 2^-27 |x|, RNE at each step: the library's split3),
    returned as one int16 tensor [3][cout][Kpad] (plane stride cout * Kpad)."""
    w = _f32(w_packed, "w")
    h = w.to(torch.bfloat16)
    r = w - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack([h, m, lo]).view(torch.int16).contiguous()


def conv2d_nhwc_planes(x, w_packed, planes, bias, cout, kh, kw, stride=1, pad=None, act="none",
                       res=None, out=None, cin=None, allow_split=False, tile=-1):
    """conv2d_nhwc with the weights also given as bf16 planes
    (split_weight_planes), as the engine runs its convs: the pre-split tiles
    (dense 1x1: the 16x16x32 conv_bf6x_kernel)."""
    _f32(x, "x")
    n, h, w, xcs = x.shape
    cin = xcs if cin is None else cin
    pad = (kh - 1) // 2 if pad is None else pad
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (w + 2 * pad - kw) // stride + 1
    if out is None:
        out = torch.empty(n, oh, ow, cout, device=x.device, dtype=torch.float32)
    d = _lib.ConvDesc(n=n, h=h, w=w, cin=cin, x_cstride=xcs, cout=cout, kh=kh, kw=kw,
                      stride=stride, pad=pad, y_cstride=out.shape[-1],
                      res_cstride=(res.shape[-1] if res is not None else 0), act=ACT[act])
    need = lib().posfeat_conv2d_workspace(ctypes.byref(d)) if allow_split else 0
    ws = torch.empty(max(need, 16), dtype=torch.uint8, device=x.device)
    check(lib().posfeat_conv2d_nhwc_planes(ctypes.byref(d), ptr(x), ptr(w_packed), ptr(planes),
                                           planes[0].numel(), ptr(bias), ptr(res), ptr(out),
                                           ptr(ws), need, tile, stream_ptr()))
    return out


def conv1x1_dual(x1, x2, w1, w2, bias1, bias2, stride2=1, act="relu", out=None):
    """y = act(x1 . w1^T + x2[:, ::s, ::s] . w2^T + bias1 + bias2) as one GEMM
    (posfeat_conv1x1_dual: a bottleneck's conv3 + downsample, the engine's
    layer1.0 / layer2.0 / layer3.0).  x1 [n, oh, ow, k1], x2 [n, h2, w2, k2]
    NHWC fp32; w1 [cout, k1], w2 [cout, k2]."""
    _f32(x1, "x1")
    _f32(x2, "x2")
    n, oh, ow, k1 = x1.shape
    _, xh, xw, k2 = x2.shape
    cout = w1.shape[0]
    planes = split_weight_planes(torch.cat([_f32(w1, "w1"), _f32(w2, "w2")], dim=1))
    bias = (_f32(bias1, "bias1") + _f32(bias2, "bias2")).contiguous()
    if out is None:
        out = torch.empty(n, oh, ow, cout, device=x1.device, dtype=torch.float32)
    check(lib().posfeat_conv1x1_dual(n, oh, ow, ptr(x1), k1, k1, ptr(x2), k2, xh, xw, stride2, k2,
                                     cout, ptr(planes), ptr(bias), ACT[act], ptr(out),
                                     out.shape[-1], stream_ptr()))
    return out


def conv2d_nhwc_instnorm_stats(x, w_packed, bias, cout, kh, kw, eps=1e-5, out=None, cin=None):
    """Conv (stride 1, 'same' pad, no act) + per-image channel mean/rstd of its
    output from the fused epilogue.  Returns (y, mean [n,cout], rstd [n,cout])."""
    _f32(x, "x")
    n, h, w, xcs = x.shape
    cin = xcs if cin is None else cin
    pad = (kh - 1) // 2
    if out is None:
        out = torch.empty(n, h, w, cout, device=x.device, dtype=torch.float32)
    d = _lib.ConvDesc(n=n, h=h, w=w, cin=cin, x_cstride=xcs, cout=cout, kh=kh, kw=kw, stride=1,
                      pad=pad, y_cstride=out.shape[-1], res_cstride=0, act=0)
    need = lib().posfeat_conv2d_stats_workspace(ctypes.byref(d))
    ws = torch.empty(max(need, 16), dtype=torch.uint8, device=x.device)
    mean = torch.empty(n, cout, device=x.device)
    rstd = torch.empty(n, cout, device=x.device)
    check(lib().posfeat_conv2d_nhwc_stats(ctypes.byref(d), ptr(x), ptr(_f32(w_packed, "w")),
                                          ptr(bias), ptr(out), ptr(ws), need, ptr(mean),
                                          ptr(rstd), float(eps), stream_ptr()))
    return out, mean, rstd


def conv2_up4_instnorm_stats(L, G, w_packed, bias, eps=1e-5, out=None):
    """KeypointDet conv2 over cat[up4(L), G] (DeteNet.py:109-112) without the
    upsampled map: L n x h x w x 192 NHWC (h = H/4), G n x H x W x 64 NHWC.
    Returns (y n x H x W x 128, mean [n,128], rstd [n,128])."""
    _f32(L, "L")
    _f32(G, "G")
    n, H, W, gcs = G.shape
    lcs = L.shape[-1]
    if out is None:
        out = torch.empty(n, H, W, 128, device=G.device, dtype=torch.float32)
    wph = torch.empty(lib().posfeat_conv2_up4_weights_floats(), device=G.device,
                      dtype=torch.float32)
    check(lib().posfeat_conv2_up4_weights(ptr(_f32(w_packed, "w")), ptr(wph), stream_ptr()))
    need = lib().posfeat_conv2_up4_workspace(n, H, W)
    ws = torch.empty(max(need, 16), dtype=torch.uint8, device=G.device)
    mean = torch.empty(n, 128, device=G.device)
    rstd = torch.empty(n, 128, device=G.device)
    check(lib().posfeat_conv2_up4(n, H, W, ptr(L), lcs, ptr(G), gcs, ptr(wph), ptr(w_packed),
                                  ptr(bias), ptr(out), out.shape[-1], ptr(ws), need, ptr(mean),
                                  ptr(rstd), float(eps), stream_ptr()))
    return out, mean, rstd


def nchw_to_nhwc(x, cstride=None):
    _f32(x, "x")
    n, c, h, w = x.shape
    cs = c if cstride is None else cstride
    y = torch.empty(n, h, w, cs, device=x.device, dtype=torch.float32)
    check(lib().posfeat_nchw_to_nhwc(ptr(x), n, c, h, w, cs, ptr(y), stream_ptr()))
    return y


def normalize_rgb8(u8):
    """uint8 [b,h,w,3] (or [h,w,3]) RGB on the device -> ImageNet-normalised
    float [b,3,h,w], bit-identical to datasets.to_input's host computation."""
    if u8.dtype != torch.uint8 or u8.shape[-1] != 3 or u8.dim() not in (3, 4):
        raise ValueError("expected uint8 [b,h,w,3]")
    if u8.dim() == 3:
        u8 = u8[None]
    u8 = u8.contiguous()
    b, h, w, _ = u8.shape
    out = torch.empty(b, 3, h, w, dtype=torch.float32, device=u8.device)
    check(lib().posfeat_normalize_rgb8(ptr(u8), b, h, w, 3 * w, ptr(out), stream_ptr()))
    return out


def nhwc_to_nchw(x, c=None):
    _f32(x, "x")
    n, h, w, cs = x.shape
    c = cs if c is None else c
    y = torch.empty(n, c, h, w, device=x.device, dtype=torch.float32)
    check(lib().posfeat_nhwc_to_nchw(ptr(x), n, c, h, w, cs, ptr(y), stream_ptr()))
    return y


class DetectWorkspace:
    """Reusable device scratch for ``detect`` (avoid per-call allocation)."""

    def __init__(self):
        self.key = None
        self.buf = None

    def get(self, b, h, w, cap, device):
        key = (b, h, w, cap, str(device))
        if key != self.key:
            n = ctypes.c_size_t()
            check(lib().posfeat_detect_workspace(b, h, w, cap, ctypes.byref(n)))
            self.buf = torch.empty(n.value, dtype=torch.uint8, device=device)
            self.key = key
        return self.buf


_DEFAULT_WS = DetectWorkspace()


def detect(kp_map, nms_radius, num_pts=False, use_nms=True, thr=False, thr_mod="mean",
           ws=None, sync=True, each=False):
    """GPU generate_kpts_single core.  kp_map: [b,1,h,w] fp32 on the GPU.

    Returns (idx [b,n] int32, coord_n [b,n,2], kp_score [b,n,1], counts [b], n).
    With ``sync=False`` the buffers are full-capacity and ``n`` is a device
    scalar tensor (no host synchronisation).  ``each=True`` (needs
    ``sync=False``): every image is selected as if detected alone and ``n`` is
    a device tensor [b] (posfeat_detect_each).
    """
    if each and sync:
        raise ValueError("each=True returns per-image counts on the device: use sync=False")
    _f32(kp_map, "kp_map")
    b, c, h, w = kp_map.shape
    if c != 1:
        raise ValueError("kp_map must have one channel")
    P = (h - 2) * (w - 2)
    if num_pts:
        cap = min(max(int(num_pts), 128), P)
    else:
        cap = P
    if thr is False or thr is None or not thr:
        mode, tval = 0, 0.0
    else:
        if thr_mod not in THR_MODE:
            raise ValueError("thr_mod must be one of %s" % list(THR_MODE))
        mode, tval = THR_MODE[thr_mod], float(thr)
    dev = kp_map.device
    idx = torch.empty(b, cap, dtype=torch.int32, device=dev)
    coord = torch.empty(b, cap, 2, dtype=torch.float32, device=dev)
    score = torch.empty(b, cap, 1, dtype=torch.float32, device=dev)
    if each:
        meta = torch.empty(2 * b, dtype=torch.int32, device=dev)  # [n_sel..., counts...]
        wsb = (ws or _DEFAULT_WS).get(b, h, w, cap, dev)
        check(lib().posfeat_detect_each(
            ptr(kp_map), b, h, w, int(nms_radius), 1 if use_nms else 0, mode, tval,
            int(num_pts) if num_pts else 0, cap, ptr(idx), ptr(coord), ptr(score), ptr(meta),
            ctypes.c_void_p(meta.data_ptr() + 4 * b), ptr(wsb), wsb.numel(), stream_ptr()))
        return idx, coord, score, meta[b:], meta[:b]
    meta = torch.empty(b + 1, dtype=torch.int32, device=dev)  # [n_sel, counts...]
    wsb = (ws or _DEFAULT_WS).get(b, h, w, cap, dev)
    check(lib().posfeat_detect(ptr(kp_map), b, h, w, int(nms_radius), 1 if use_nms else 0, mode,
                               tval, int(num_pts) if num_pts else 0, cap, ptr(idx), ptr(coord),
                               ptr(score), ptr(meta), ctypes.c_void_p(meta.data_ptr() + 4),
                               ptr(wsb), wsb.numel(), stream_ptr()))
    counts = meta[1:]
    if not sync:
        return idx, coord, score, counts, meta[:1]
    n = int(meta[0].item())
    return idx[:, :n], coord[:, :n], score[:, :n], counts, n


def nms_mask(score, radius):
    """score [b,1,h,w] -> bool mask [b,1,h,w] (reference nms tie rule)."""
    _f32(score, "score")
    b, c, h, w = score.shape
    if c != 1:
        raise ValueError("score must have one channel")
    m = torch.empty(b, 1, h, w, dtype=torch.uint8, device=score.device)
    check(lib().posfeat_nms_mask(ptr(score), b, h, w, int(radius), ptr(m), stream_ptr()))
    return m.bool()


def sample_desc_nhwc(fmap_nhwc, coord_n, c=None, normalize=True, n_valid=None, each=False):
    """Bilinear (align_corners=False, zeros) sampling of an NHWC map at coord_n [b,n,2].
    ``n_valid``: device int32, one count for the batch, or ``each=True`` one per
    image ([b], posfeat_sample_desc_each); rows past the count are zeros."""
    _f32(fmap_nhwc, "fmap")
    coord_n = _f32(coord_n.contiguous(), "coord_n")
    b, h, w, cs = fmap_nhwc.shape
    c = cs if c is None else c
    npts = coord_n.shape[1]
    out = torch.empty(b, npts, c, device=fmap_nhwc.device, dtype=torch.float32)
    if each:
        if n_valid is None or n_valid.numel() != b or n_valid.dtype != torch.int32:
            raise ValueError("each=True needs n_valid: int32 [b] on the device")
        check(lib().posfeat_sample_desc_each(ptr(fmap_nhwc), b, c, h, w, cs, ptr(coord_n), npts,
                                             ptr(n_valid), 1 if normalize else 0, ptr(out),
                                             stream_ptr()))
        return out
    check(lib().posfeat_sample_desc(ptr(fmap_nhwc), b, c, h, w, cs, ptr(coord_n), npts,
                                    ptr(n_valid), 1 if normalize else 0, ptr(out), stream_ptr()))
    return out


def sample_desc_strided(fmap_base, b, c, h, w, cs, coord_n, normalize=True, n_valid=None):
    """Same, on a raw NHWC pointer owned by the engine workspace."""
    coord_n = _f32(coord_n.contiguous(), "coord_n")
    npts = coord_n.shape[1]
    out = torch.empty(b, npts, c, device=coord_n.device, dtype=torch.float32)
    check(lib().posfeat_sample_desc(ctypes.c_void_p(fmap_base), b, c, h, w, cs, ptr(coord_n),
                                    npts, ptr(n_valid), 1 if normalize else 0, ptr(out),
                                    stream_ptr()))
    return out
