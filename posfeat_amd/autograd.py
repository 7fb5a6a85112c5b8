"""Autograd bindings of the HIP training paths to the torch modules -- the
reference Trainer's plug points (managers/trainer.py:296-331):

    model.set_eval(); getattr(model, m).train() for m in optimal_modules
    outputs = model.forward(inputs)          # differentiable maps
    processed = preprocess(inputs, outputs)  # Preprocess_Line2Window / Skip
    loss, _ = loss_module(inputs, outputs, processed)
    optimizer.zero_grad(); loss.backward(); optimizer.step()

* keypoint training (configs/train_kp.yaml, optimal_modules ['localheader']):
  ``HeadBinding`` keeps the packed KeypointDet region of an
  ``ExtractionEngine(train=True)`` in step with ``model.localheader``'s
  parameters; the engine's ``local_point`` is returned through ``HeadFn``,
  whose backward is ``posfeat_model_head_backward`` (dL/d packed head
  params), laid back out per parameter on the device.
* descriptor training (configs/train_desc.yaml, optimal_modules
  ['backbone']): ``BackboneBinding`` drives a ``training.BackboneTrainer``
  (train-mode BatchNorm, running statistics) from ``model.backbone``'s
  parameters and buffers; ``local_map`` is returned through ``BackboneFn``,
  whose backward is ``posfeat_bbtrain_backward``.  The updated running
  statistics are written back into the module's buffers after every forward
  (and num_batches_tracked advanced), as torch's BatchNorm does.

Packing/unpacking between torch's [cout, cin, kh, kw] and the kernels'
[cout][Kpad] layout is a device-side permute (weights.pack_conv's order);
under DDP (``model.set_parallel``) the packed gradient is all-reduced once
(mean over ranks) before it is unpacked -- one RCCL call per module per
step instead of DDP's per-bucket calls.
"""
import torch

from . import weights


def pack_conv_t(w, kpad):
    """torch [cout, cin, kh, kw] -> [cout, kpad] in weights.pack_conv's K order."""
    cout, cin, kh, kw = w.shape
    cinp = (cin + 3) // 4 * 4
    k = kh * kw * cinp
    out = w.new_zeros(cout, kpad)
    if cin % 32 == 0:
        out[:, :k] = w.reshape(cout, cin // 32, 32, kh, kw).permute(0, 1, 3, 4, 2).reshape(cout, k)
    else:
        t = w.new_zeros(cout, kh, kw, cinp)
        t[..., :cin] = w.permute(0, 2, 3, 1)
        out[:, :k] = t.reshape(cout, k)
    return out


def unpack_conv_t(wp, cout, cin, kh, kw):
    """Inverse of pack_conv_t: [cout][kpad] (flat or 2-D) -> [cout, cin, kh, kw]."""
    cinp = (cin + 3) // 4 * 4
    k = kh * kw * cinp
    wp = wp.reshape(cout, -1)[:, :k]
    # always a copy: for 1x1 convs the permutation is the identity and a
    # reshape would alias the packed buffer (which the next backward reuses)
    if cin % 32 == 0:
        t = wp.reshape(cout, cin // 32, kh, kw, 32).permute(0, 1, 4, 2, 3)
    else:
        t = wp.reshape(cout, kh, kw, cinp)[..., :cin].permute(0, 3, 1, 2)
    return t.clone(memory_format=torch.contiguous_format).reshape(cout, cin, kh, kw)


def _mean_over_ranks(buf, parallel):
    if parallel:
        from .parallel import allreduce_head_grad
        scale = allreduce_head_grad(buf)
        if scale != 1.0:
            buf.mul_(scale)
    return buf


class _Binding:
    """items: (tensor, kind, offset, info) mapping module tensors to a blob."""

    def __init__(self):
        self.items = []
        self.params = []
        self._key = None
        self.token = 0
        self.parallel = False

    def _versions(self):
        return tuple(t._version for t, _, _, _ in self.items)

    def pack_into(self, blob):
        with torch.no_grad():
            for t, kind, off, info in self.items:
                src = t.detach().to(blob.device, torch.float32)
                if kind == "w":
                    cout, cin, kh, kw, kpad = info
                    blob[off:off + cout * kpad].view(cout, kpad).copy_(pack_conv_t(src, kpad))
                else:
                    blob[off:off + src.numel()].copy_(src.reshape(-1))

    def grads(self, gp):
        out = []
        for t, kind, off, info in self.items:
            if kind == "w":
                cout, cin, kh, kw, kpad = info
                g = unpack_conv_t(gp[off:off + cout * kpad], cout, cin, kh, kw)
            else:
                g = gp[off:off + t.numel()].clone().reshape(t.shape)
            out.append(g.to(t.device, t.dtype))
        return out


class HeadBinding(_Binding):
    def __init__(self, engine, module):
        super().__init__()
        self.engine = engine
        specs = engine.specs
        hoff = weights.head_offset(specs)
        sd = module.state_dict(keep_vars=True)
        for name, cout, cin, kh, kw, w_off, b_off in specs:
            if not name.startswith("head."):
                continue
            if name == "head.prelu":
                self.items.append((sd["relu.weight"], "v", b_off - hoff, None))
                continue
            _, wk, bk, _ = weights.conv_sources(name)
            kpad = weights.packed_k(cin, kh, kw)[2]
            self.items.append((sd[wk], "w", w_off - hoff, (cout, cin, kh, kw, kpad)))
            self.items.append((sd[bk], "v", b_off - hoff, None))
        self.params = [t for t, _, _, _ in self.items]

    def sync(self):
        key = self._versions()
        if key != self._key:
            self.pack_into(self.engine.head_weights())
            self._key = key

    def backward(self, dlp):
        gp = self.engine.head_backward(dlp.contiguous())
        return self.grads(_mean_over_ranks(gp, self.parallel))


class HeadFn(torch.autograd.Function):
    """local_point of the last engine run; backward = the head backward kernels."""

    @staticmethod
    def forward(ctx, lp, binding, token, *params):
        ctx.binding, ctx.token = binding, token
        return lp.clone()

    @staticmethod
    def backward(ctx, g):
        b = ctx.binding
        if b.token != ctx.token:
            raise RuntimeError("the keypoint-training engine ran again between this forward and "
                               "its backward (its intermediates are per run)")
        return (None, None, None, *b.backward(g))


class BackboneBinding(_Binding):
    """model.backbone (ResUNet param holder) <-> a BackboneTrainer of one shape."""

    def __init__(self, module, batch, h, w, device):
        super().__init__()
        from .training import BackboneTrainer
        self.module = module
        sd = module.state_dict(keep_vars=True)
        self.trainer = BackboneTrainer({k: v.detach() for k, v in sd.items()}, batch, h, w,
                                       device=device)
        layers, _, _ = self.trainer.table
        self.stat_items = []
        self.nbt = []
        for name, cin, cout, k, stride, has_bias, offs in layers:
            _, wk, bk, bn = weights.conv_sources(name)
            kpad = weights.packed_k(cin, k, k)[2]
            self.items.append((sd[wk], "w", offs[0], (cout, cin, k, k, kpad)))
            if has_bias:
                self.items.append((sd[bk], "v", offs[1], None))
            self.items.append((sd[bn + ".weight"], "v", offs[2], None))
            self.items.append((sd[bn + ".bias"], "v", offs[3], None))
            self.stat_items.append((sd[bn + ".running_mean"], offs[4]))
            self.stat_items.append((sd[bn + ".running_var"], offs[5]))
            self.nbt.append(sd[bn + ".num_batches_tracked"])
        self.params = [t for t, _, _, _ in self.items]
        # global_map's conv_coarse takes no part in the descriptor loss: the
        # reference leaves its .grad None (DDP find_unused_parameters)
        self.unused = [name.startswith("conv_coarse") for name, *_ in layers
                       for _ in range(4 if _has_bias(layers, name) else 3)]
        self.tokens = [0, 0]
        self._key = self._versions()       # the trainer was built from these values
        self._skey = self._stat_versions()

    def _stat_versions(self):
        return tuple(t._version for t, _ in self.stat_items)

    def sync(self):
        key = self._versions()
        if key != self._key:
            self.pack_into(self.trainer.params)
            self._key = key
        if self._stat_versions() != self._skey:   # buffers changed outside (e.g. loaded)
            with torch.no_grad():
                for t, off in self.stat_items:
                    self.trainer.stats[off:off + t.numel()].copy_(t.detach().reshape(-1))

    def forward(self, img, slot):
        self.sync()
        lm = self.trainer.forward(img, slot)
        with torch.no_grad():                     # BatchNorm's running-statistics update
            st = self.trainer.stats
            for t, off in self.stat_items:
                t.copy_(st[off:off + t.numel()].view(t.shape).to(t.device))
            for t in self.nbt:
                t.add_(1)
        self._skey = self._stat_versions()
        self.tokens[slot] += 1
        return lm

    def backward(self, dlm_nhwc, slot):
        self.trainer.backward(dlm_nhwc, slot, accumulate=False)
        gs = self.grads(_mean_over_ranks(self.trainer.grad, self.parallel))
        return [None if u else g for g, u in zip(gs, self.unused)]


def _has_bias(layers, name):
    return next(hb for n, _, _, _, _, hb, _ in layers if n == name)


class BackboneFn(torch.autograd.Function):
    """NCHW local_map of one BackboneTrainer slot; backward = the backbone
    backward kernels (dL/d params of ResUNet through train-mode BatchNorm)."""

    @staticmethod
    def forward(ctx, lm_nchw, binding, slot, token, *params):
        ctx.binding, ctx.slot, ctx.token = binding, slot, token
        return lm_nchw.clone()

    @staticmethod
    def backward(ctx, g):
        from . import ops
        b = ctx.binding
        if b.tokens[ctx.slot] != ctx.token:
            raise RuntimeError("the backbone ran again between this forward and its backward")
        d = ops.nchw_to_nhwc(g.float().contiguous())
        return (None, None, None, None, *b.backward(d, ctx.slot))
