"""Parameter layout, seeded weight recipe, checkpoint I/O and device packing.

The reference stores one ``state_dict`` per module (``backbone.pth`` and
``localheader.pth``; networks/PoSFeat_model.py:57-81).  The effective
extraction model is ``ResUNet(encoder='resnet50', coarse_out_ch=128,
fine_out_ch=128)`` (networks/DescNet.py:12-48) with a torchvision ResNet-50
encoder cut after ``layer3`` (DescNet.py:27-35), plus
``KeypointDet(in_channels=192, out_channels=1, prior='identity',
act='Softplus')`` (networks/DeteNet.py:9-22; configs/train_desc.yaml:16-31).

This module owns three things:

* ``backbone_param_shapes()`` / ``head_param_shapes()`` -- the exact key order
  and shapes of those two state dicts (300 + 9 keys);
* ``seeded_state_dicts(seed)`` -- the deterministic random-weight recipe used by
  tests, fixtures and the benchmark (no pretrained download, no checkpoint in
  the container): every tensor comes from ``numpy.random.RandomState(base+i)``
  so it is bit-stable across machines;
* ``pack_for_device(...)`` -- eval-mode BatchNorm folding and the packed
  ``[Cout][KH][KW][Cin_pad]`` weight blob the HIP engine consumes.  The layer
  table it follows is read from the C-ABI (``posfeat_model_conv_spec``) so the
  packing order has a single source of truth.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

BN_EPS = 1e-5

# torchvision ResNet-50 (Bottleneck, expansion 4, stride on the 3x3 conv) cut
# after layer3, as ResUNet uses it (DescNet.py:23-35).
_RESNET_LAYERS = (("layer1", 64, 3, 1), ("layer2", 128, 4, 2), ("layer3", 256, 6, 2))
# ResUNet decoder modules (DescNet.py:37-47): name, cin, cout, kernel
_DECODER = (("conv_coarse", 1024, 128, 1), ("upconv3.conv", 1024, 512, 3),
            ("iconv3", 1024, 512, 3), ("upconv2.conv", 512, 256, 3),
            ("iconv2", 512, 256, 3), ("conv_fine", 256, 128, 1))


def _bn(prefix, c):
    return [(prefix + ".weight", (c,)), (prefix + ".bias", (c,)),
            (prefix + ".running_mean", (c,)), (prefix + ".running_var", (c,)),
            (prefix + ".num_batches_tracked", ())]


def backbone_param_shapes():
    """Ordered (key, shape) list of the ResUNet state dict (300 entries)."""
    out = [("firstconv.weight", (64, 3, 7, 7))] + _bn("firstbn", 64)
    inplanes = 64
    for lname, planes, blocks, stride in _RESNET_LAYERS:
        for bi in range(blocks):
            p = "%s.%d" % (lname, bi)
            out.append((p + ".conv1.weight", (planes, inplanes, 1, 1)))
            out += _bn(p + ".bn1", planes)
            out.append((p + ".conv2.weight", (planes, planes, 3, 3)))
            out += _bn(p + ".bn2", planes)
            out.append((p + ".conv3.weight", (planes * 4, planes, 1, 1)))
            out += _bn(p + ".bn3", planes * 4)
            if bi == 0:
                out.append((p + ".downsample.0.weight", (planes * 4, inplanes, 1, 1)))
                out += _bn(p + ".downsample.1", planes * 4)
            inplanes = planes * 4
    for name, cin, cout, k in _DECODER:
        out.append((name + ".conv.weight", (cout, cin, k, k)))
        out.append((name + ".conv.bias", (cout,)))
        out += _bn(name + ".bn", cout)
    return out


def head_param_shapes(in_channels=192, out_channels=1):
    """Ordered (key, shape) list of the KeypointDet state dict (DeteNet.py:9-22)."""
    return [("conv1.weight", (in_channels, in_channels, 3, 3)), ("conv1.bias", (in_channels,)),
            ("conv2.weight", (128, in_channels + 64, 3, 3)), ("conv2.bias", (128,)),
            ("conv3.weight", (out_channels, 128, 1, 1)), ("conv3.bias", (out_channels,)),
            ("relu.weight", (1,)),
            ("convimg.weight", (64, 3, 3, 3)), ("convimg.bias", (64,))]


def _draw(rs, key, shape):
    if key.endswith("num_batches_tracked"):
        return np.array(0, dtype=np.int64)
    if key == "relu.weight":                       # nn.PReLU() init
        return np.full(shape, 0.25, dtype=np.float32)
    if len(shape) == 4:                            # conv weight, He-scaled
        fan_in = shape[1] * shape[2] * shape[3]
        return (rs.standard_normal(shape) * math.sqrt(2.0 / fan_in)).astype(np.float32)
    if key.endswith("running_mean"):
        return rs.normal(0.0, 0.1, shape).astype(np.float32)
    if key.endswith("running_var"):
        return rs.uniform(0.5, 1.5, shape).astype(np.float32)
    if key.endswith("bn3.weight"):
        # small residual-branch gain keeps the 13-block ResNet stack O(1)
        # (otherwise random running stats let activations grow ~2x per block)
        return rs.uniform(0.1, 0.3, shape).astype(np.float32)
    if ".bn" in key or "bn1" in key or "bn2" in key or "bn3" in key or "firstbn" in key \
            or "downsample.1" in key:
        if key.endswith(".weight"):
            return rs.uniform(0.5, 1.5, shape).astype(np.float32)
        return rs.normal(0.0, 0.1, shape).astype(np.float32)
    # conv bias
    return rs.uniform(-0.1, 0.1, shape).astype(np.float32)


def seeded_state_dicts(seed=0, as_torch=True, parts=("backbone", "localheader")):
    """Deterministic random weights for (backbone, localheader).

    Tensor i of the backbone comes from ``RandomState(seed*100003 + i)``,
    tensor i of the head from ``RandomState(seed*100003 + 50000 + i)``.
    ``parts``: which of the two to draw (the other is returned as None; the
    values of a drawn part do not depend on it).
    """
    base = seed * 100003
    bb = hd = None
    if "backbone" in parts:
        bb = OrderedDict()
        for i, (k, s) in enumerate(backbone_param_shapes()):
            bb[k] = _draw(np.random.RandomState(base + i), k, s)
    if "localheader" in parts:
        hd = OrderedDict()
        for i, (k, s) in enumerate(head_param_shapes()):
            hd[k] = _draw(np.random.RandomState(base + 50000 + i), k, s)
    if as_torch:
        import torch
        conv = lambda d: None if d is None else OrderedDict(
            (k, torch.from_numpy(np.ascontiguousarray(v))) for k, v in d.items())
        bb, hd = conv(bb), conv(hd)
    return bb, hd


# Deferred seeding: modules built inside ``deferred_seed()`` skip the seeded
# draw (20.5 M normal draws for the backbone, ~0.25 s on the GPU box's host)
# and mark themselves pending; ``materialize_seed`` draws it later unless a
# checkpoint replaced every tensor first (PoSFeat.load_checkpoint,
# Extractor: the reference flow always loads one right after construction).
_DEFER = [0]


class deferred_seed:
    def __enter__(self):
        _DEFER[0] += 1
        return self

    def __exit__(self, *exc):
        _DEFER[0] -= 1
        return False


def seed_deferred():
    return _DEFER[0] > 0


def seed_module(module, part):
    """Load the seeded recipe's ``part`` into ``module`` now, or mark it
    pending inside ``deferred_seed()``."""
    if seed_deferred():
        module._seed_pending = part
        return
    bb, hd = seeded_state_dicts(0, parts=(part,))
    module.load_state_dict(bb if part == "backbone" else hd)
    module._seed_pending = None


def materialize_seed(module):
    part = getattr(module, "_seed_pending", None)
    if part:
        bb, hd = seeded_state_dicts(0, parts=(part,))
        module.load_state_dict(bb if part == "backbone" else hd)
        module._seed_pending = None


def seeded_image(i, h=480, w=640):
    """Synthetic ImageNet-normalised input (datasets/hpatches.py:14-17).

    uint8 ``RandomState(1000+i).randint(0,256,(h,w,3))`` -> /255 -> mean/std
    normalise -> float32 ``3 x h x w``.
    """
    rs = np.random.RandomState(1000 + i)
    im = rs.randint(0, 256, (h, w, 3)).astype(np.float32) / np.float32(255.0)
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    im = (im - mean) / std
    return np.ascontiguousarray(im.transpose(2, 0, 1).astype(np.float32))


def strip_ddp_prefix(sd):
    """DDP-saved checkpoints carry ``module.`` (PoSFeat_model.py:50-55, 74-81)."""
    out = OrderedDict()
    for k, v in sd.items():
        out[k[7:] if k.startswith("module.") else k] = v
    return out


def load_checkpoint_dir(path):
    """Load ``backbone.pth`` / ``localheader.pth`` like PoSFeat.load_checkpoint
    (PoSFeat_model.py:57-72), but never executing pickled code."""
    import os
    import torch
    out = {}
    for name in ("backbone", "localheader"):
        p = os.path.join(str(path), name + ".pth")
        if os.path.exists(p):
            out[name] = strip_ddp_prefix(torch.load(p, map_location="cpu", weights_only=True))
        else:
            out[name] = None
    return out["backbone"], out["localheader"]


def _np(v):
    try:
        return v.detach().cpu().numpy()
    except AttributeError:
        return np.asarray(v)


def fold_conv(sd, conv_w, conv_b=None, bn=None):
    """Return (W[Cout,Cin,KH,KW] float64, b[Cout] float64) with eval-BN folded.

    conv(x)*g/sqrt(v+eps) + (b - m)*g/sqrt(v+eps) + beta  (torch batch_norm eval).
    """
    w = _np(sd[conv_w]).astype(np.float64)
    b = _np(sd[conv_b]).astype(np.float64) if conv_b is not None else np.zeros(w.shape[0])
    if bn is not None:
        g = _np(sd[bn + ".weight"]).astype(np.float64)
        beta = _np(sd[bn + ".bias"]).astype(np.float64)
        m = _np(sd[bn + ".running_mean"]).astype(np.float64)
        v = _np(sd[bn + ".running_var"]).astype(np.float64)
        s = g / np.sqrt(v + BN_EPS)
        w = w * s[:, None, None, None]
        b = (b - m) * s + beta
    return w, b


def conv_sources(name):
    """Map an engine conv name (C-ABI spec) to (module, weight, bias, bn) keys."""
    if name.startswith("head."):
        n = name[5:]
        return "localheader", n + ".weight", n + ".bias", None
    if name == "firstconv":
        return "backbone", "firstconv.weight", None, "firstbn"
    if name.startswith("layer"):
        # layerX.Y.convZ  |  layerX.Y.downsample
        if name.endswith("downsample"):
            return "backbone", name + ".0.weight", None, name + ".1"
        idx = name[-1]
        return "backbone", name + ".weight", None, name[:-5] + "bn" + idx
    return "backbone", name + ".conv.weight", name + ".conv.bias", name + ".bn"


def packed_k(cin, kh, kw):
    cinp = (cin + 3) // 4 * 4
    k = kh * kw * cinp
    return cinp, k, (k + 31) // 32 * 32


def pack_conv(w, b):
    """[Cout,Cin,KH,KW] -> float32 [Cout][Kpad].

    K order (must match conv.hip): (cin/32, kh, kw, cin%32) when Cin % 32 == 0,
    else (kh, kw, cin padded to 4) zero-padded to a multiple of 32."""
    cout, cin, kh, kw = w.shape
    cinp, k, kpad = packed_k(cin, kh, kw)
    out = np.zeros((cout, kpad), np.float32)
    if cin % 32 == 0:
        wp = w.reshape(cout, cin // 32, 32, kh, kw).transpose(0, 1, 3, 4, 2)
        out[:, :k] = wp.reshape(cout, k)
    else:
        wp = np.zeros((cout, kh, kw, cinp), np.float64)
        wp[:, :, :, :cin] = w.transpose(0, 2, 3, 1)
        out[:, :k] = wp.reshape(cout, k)
    return out, b.astype(np.float32)


def unpack_conv(wp, cout, cin, kh, kw):
    """Inverse of ``pack_conv`` for the weight: [Cout][Kpad] -> [Cout,Cin,KH,KW]."""
    cinp, k, kpad = packed_k(cin, kh, kw)
    wp = np.asarray(wp, np.float32).reshape(cout, kpad)[:, :k]
    if cin % 32 == 0:
        return np.ascontiguousarray(
            wp.reshape(cout, cin // 32, kh, kw, 32).transpose(0, 1, 4, 2, 3).reshape(cout, cin, kh, kw))
    return np.ascontiguousarray(wp.reshape(cout, kh, kw, cinp)[..., :cin].transpose(0, 3, 1, 2))


def head_offset(specs):
    """First float of the KeypointDet region of the blob (the head specs are
    the contiguous tail of the engine's layer table)."""
    return min(s[5] for s in specs if s[0].startswith("head."))


def pack_head(head_sd, specs, total, head_prelu_key="relu.weight"):
    """The KeypointDet part of the blob (floats [head_offset, total)) from a
    head state dict -- also used to lay reference gradients out like the
    engine's packed gradient buffer."""
    hoff = head_offset(specs)
    out = np.zeros(total - hoff, np.float32)
    for name, cout, cin, kh, kw, w_off, b_off in specs:
        if not name.startswith("head."):
            continue
        if name == "head.prelu":
            out[b_off - hoff] = float(_np(head_sd[head_prelu_key]).reshape(-1)[0])
            continue
        _, wk, bk, _ = conv_sources(name)
        wp, bp = pack_conv(_np(head_sd[wk]).astype(np.float64), _np(head_sd[bk]).astype(np.float64))
        out[w_off - hoff:w_off - hoff + wp.size] = wp.reshape(-1)
        out[b_off - hoff:b_off - hoff + cout] = bp
    return out


def unpack_head(region, specs, head_prelu_key="relu.weight"):
    """Head state dict (KeypointDet key order, DeteNet.py:9-22) from the blob's
    head region -- PoSFeat.save_checkpoint's localheader.pth after training."""
    hoff = head_offset(specs)
    region = np.asarray(region, np.float32)
    vals = {}
    for name, cout, cin, kh, kw, w_off, b_off in specs:
        if not name.startswith("head."):
            continue
        if name == "head.prelu":
            vals[head_prelu_key] = region[b_off - hoff:b_off - hoff + 1].copy()
            continue
        _, wk, bk, _ = conv_sources(name)
        kpad = packed_k(cin, kh, kw)[2]
        vals[wk] = unpack_conv(region[w_off - hoff:w_off - hoff + cout * kpad], cout, cin, kh, kw)
        vals[bk] = region[b_off - hoff:b_off - hoff + cout].copy()
    return OrderedDict((k, vals[k]) for k, _ in head_param_shapes())


def pack_for_device(backbone_sd, head_sd, specs, head_prelu_key="relu.weight"):
    """Build the flat float32 weight blob in the order of ``specs``.

    ``specs``: list of (name, cout, cin, kh, kw, w_off, b_off) from the C-ABI
    (offsets in floats).  Returns a 1-D float32 numpy array.  The PReLU
    scalar is written at the end (offset given by the last spec entry named
    ``head.prelu``).
    """
    total = 0
    for s in specs:
        total = max(total, s[6] + max(s[1], 1))
    blob = np.zeros(total, np.float32)
    mods = {"backbone": backbone_sd, "localheader": head_sd}
    for name, cout, cin, kh, kw, w_off, b_off in specs:
        if name == "head.prelu":
            blob[b_off] = float(_np(head_sd[head_prelu_key]).reshape(-1)[0])
            continue
        mod, wk, bk, bn = conv_sources(name)
        sd = mods[mod]
        w, b = fold_conv(sd, wk, bk, bn)
        if w.shape != (cout, cin, kh, kw):
            raise ValueError("weight %s has shape %s, engine expects %s"
                             % (wk, w.shape, (cout, cin, kh, kw)))
        wp, bp = pack_conv(w, b)
        blob[w_off:w_off + wp.size] = wp.reshape(-1)
        blob[b_off:b_off + cout] = bp
    return blob


# ----------------------------------------------------------------------------
# Train-mode backbone (configs/train_desc.yaml): raw conv weights + BatchNorm
# affine parameters in one blob, running statistics in a second one (the C-ABI
# table posfeat_bbtrain_layer gives the offsets; _lib.bbtrain_table()).
def pack_bbtrain(sd, table):
    """(params, stats) float32 blobs from a ResUNet state dict (DescNet.py key
    names).  Conv weights are packed like ``pack_conv``; the gradient blob the
    backward writes has the params layout."""
    layers, npar, nst = table
    params = np.zeros(npar, np.float32)
    stats = np.zeros(nst, np.float32)
    for name, cin, cout, k, stride, has_bias, offs in layers:
        _, wk, bk, bn = conv_sources(name)
        w = _np(sd[wk]).astype(np.float64)
        if w.shape != (cout, cin, k, k):
            raise ValueError("weight %s has shape %s, expected %s" % (wk, w.shape, (cout, cin, k, k)))
        b = _np(sd[bk]).astype(np.float64) if has_bias else np.zeros(cout)
        wp, bp = pack_conv(w, b)
        params[offs[0]:offs[0] + wp.size] = wp.reshape(-1)
        if has_bias:
            params[offs[1]:offs[1] + cout] = bp
        params[offs[2]:offs[2] + cout] = _np(sd[bn + ".weight"])
        params[offs[3]:offs[3] + cout] = _np(sd[bn + ".bias"])
        stats[offs[4]:offs[4] + cout] = _np(sd[bn + ".running_mean"])
        stats[offs[5]:offs[5] + cout] = _np(sd[bn + ".running_var"])
    return params, stats


def unpack_bbtrain(params, table, stats=None, num_batches_tracked=None):
    """Inverse of ``pack_bbtrain``: an OrderedDict in the ResUNet state-dict key
    order (``backbone_param_shapes``).  With ``stats`` it is a full
    ``backbone.pth`` (PoSFeat.save_checkpoint, PoSFeat_model.py:74-81);
    without, only the trainable tensors (e.g. a gradient blob)."""
    layers, _, _ = table
    params = np.asarray(params, np.float32)
    vals = {}
    for name, cin, cout, k, stride, has_bias, offs in layers:
        _, wk, bk, bn = conv_sources(name)
        kpad = packed_k(cin, k, k)[2]
        vals[wk] = unpack_conv(params[offs[0]:offs[0] + cout * kpad], cout, cin, k, k)
        if has_bias:
            vals[bk] = params[offs[1]:offs[1] + cout].copy()
        vals[bn + ".weight"] = params[offs[2]:offs[2] + cout].copy()
        vals[bn + ".bias"] = params[offs[3]:offs[3] + cout].copy()
        if stats is not None:
            st = np.asarray(stats, np.float32)
            vals[bn + ".running_mean"] = st[offs[4]:offs[4] + cout].copy()
            vals[bn + ".running_var"] = st[offs[5]:offs[5] + cout].copy()
            vals[bn + ".num_batches_tracked"] = np.array(int(num_batches_tracked or 0), np.int64)
    return OrderedDict((k, vals[k]) for k, _ in backbone_param_shapes() if k in vals)
