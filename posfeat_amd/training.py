"""Keypoint-head training step on MI355X (config 5 of BASELINE.json).

Reference: one inner iteration of ``Trainer.train`` (managers/trainer.py:286-356)
with configs/train_kp.yaml -- ``optimal_modules: ['localheader']``, SGD lr 1e-3,
``losses: ['DiskLoss']``, no preprocess (``Preprocess_Skip``):

    outputs = model.forward(inputs)            # extract(im1), extract(im2); the
                                               # backbone is frozen (eval BN) and
                                               # its maps are detached (PoSFeat_model.py:97-102)
    loss, _ = DiskLoss(inputs, outputs, None)  # losses/kploss.py:132-197
    optimizer.zero_grad(); loss.backward()     # -> localheader grads (DeteNet.py)
    [DDP: gradient all-reduce, mean over ranks] optimizer.step()

Here: ONE engine forward over the 2b images (im1 then im2 -- instance norm is
per image, so batching the pair is exact), ``posfeat_disk_loss_grad`` (loss +
dL/d score maps), ``posfeat_model_head_backward`` (dL/d head params in the
packed blob layout), one RCCL all-reduce of that 2.5 MB buffer when world > 1,
and ``posfeat_sgd`` on the head region of the device weight blob.  Every byte
of arithmetic is in libposfeat_hip.so; torch provides memory, the RNG for the
sampling uniforms and ``torch.distributed``.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import c_int, check, lib, ptr, stream_ptr
from .engine import ExtractionEngine, _load_tile_db
from .parallel import allreduce_head_grad

DISK_DEFAULTS = {"grid_size": 8, "loss_distance": "cos", "temperature_base": 60,
                 "temperature_max": 60, "epipolar_reward": "constant_reward",
                 "reward_config": {"reward_thr": 2, "rescale_thr": False}, "cor_detach": True,
                 "good_reward": 1, "bad_reward": -0.25, "kp_penalty": -0.001,
                 "match_grad": False}


# configs/train_desc.yaml:61-91 (preprocess_train_config, EpipolarLoss_full_config)
DESC_PRE_DEFAULTS = {"kps_generator": "generate_kpts_regular_grid_random",
                     "kps_generator_config": {"grid_size": 16, "map_init": "identity",
                                              "keep_spatial": True, "random_select": "random"},
                     "window_size": 0.1, "loss_distance": "cos", "use_nn_grid": False,
                     "use_line_search": True,
                     "line_search_config": {"line_step": 100, "use_nn": True, "loc_rand": True},
                     "temperature_base": 60, "temperature_max": 60}
DESC_EPI_DEFAULTS = {"grid_cost_thr": 0.5, "win_cost_thr": 0.1, "use_std_as_weight": True,
                     "weight_grid": 0, "weight_window": 1}


def _check_disk_config(cfg):
    rc = cfg.get("reward_config", {})
    if (cfg["grid_size"] != 8 or cfg["epipolar_reward"] != "constant_reward"
            or rc.get("rescale_thr", False) or cfg.get("loss_distance", "cos") != "cos"
            or not cfg.get("cor_detach", True) or cfg.get("match_grad", False)):
        raise NotImplementedError("posfeat_amd implements the configs/train_kp.yaml DiskLoss "
                                  "(grid 8, constant_reward, cor_detach, no match_grad)")


class KeypointTrainStep:
    """``step(im1, im2, F1, F2, epoch)`` = forward + DiskLoss + backward +
    (all-reduce) + SGD for one batch of b image pairs per rank."""

    def __init__(self, engine: ExtractionEngine, disk_config=None, lr=1e-3, group=None):
        if not engine.train:
            raise ValueError("KeypointTrainStep needs ExtractionEngine(train=True)")
        self.engine = engine
        self.cfg = dict(DISK_DEFAULTS if disk_config is None else disk_config)
        _check_disk_config(self.cfg)
        self.lr = float(lr)
        self.group = group
        self._ws = {}
        self._grad = None

    def _workspace(self, b, h, w, dev):
        key = (b, h, w)
        if key not in self._ws:
            need = lib().posfeat_disk_loss_grad_workspace(b, h, w)
            if need == 0:
                raise ValueError("image size must be a multiple of 8")
            self._ws[key] = torch.empty(need, dtype=torch.uint8, device=dev)
        return self._ws[key]

    def loss_and_grad(self, kp, lmap_nhwc, F1, F2, epoch=1, draws=None):
        """DiskLoss value (out[4] = loss, reinforce, kp_penalty, n_kps) and dL/d kp
        for kp = cat[kp1, kp2] ([2b,1,H,W]) and the engine's NHWC local maps."""
        b2, _, H, W = kp.shape
        b = b2 // 2
        dev = kp.device
        T = float(min(self.cfg["temperature_base"] + epoch, self.cfg["temperature_max"]))
        n = (H // 8) * (W // 8)
        cs = lmap_nhwc.shape[-1]
        if draws is None:
            uni = torch.rand(2, b, n, 65, device=dev)
            u1, u2 = uni[0], uni[1]
            p1 = p2 = a1 = a2 = None
        else:
            p1, p2, a1, a2 = [d.to(dev).reshape(b, n).contiguous() for d in draws]
            p1, p2 = p1.int(), p2.int()
            a1, a2 = a1.to(torch.uint8), a2.to(torch.uint8)
            u1 = u2 = None
        ws = self._workspace(b, H, W, dev)
        out = torch.empty(4, device=dev)
        dkp = torch.empty_like(kp)
        rc = self.cfg.get("reward_config", {})
        check(lib().posfeat_disk_loss_grad(
            ptr(kp[:b]), ptr(kp[b:]), ptr(lmap_nhwc[:b]), cs, ptr(lmap_nhwc[b:]), cs, b, H, W,
            ptr(F1), ptr(F2), ptr(p1), ptr(p2), ptr(a1), ptr(a2), ptr(u1), ptr(u2), T,
            float(rc.get("reward_thr", 2)), float(self.cfg["good_reward"]),
            float(self.cfg["bad_reward"]), float(self.cfg["kp_penalty"]), ptr(out), ptr(dkp[:b]),
            ptr(dkp[b:]), ptr(ws), ws.numel(), stream_ptr()))
        return out, dkp

    def step(self, im1, im2, F1, F2, epoch=1, draws=None, update=True):
        """Returns (out[4], grad) -- grad is the (all-reduced, summed) packed head
        gradient; the SGD update uses lr / world (DDP's mean over ranks)."""
        _lib.require_device(im1)
        b = im1.shape[0]
        imgs = torch.cat([im1, im2], 0).float().contiguous()
        res = self.engine.run(imgs, outputs=())
        F1 = F1.to(imgs.device).float().contiguous()
        F2 = F2.to(imgs.device).float().contiguous()
        out, dkp = self.loss_and_grad(res["local_point"], res["_local_map_nhwc"], F1, F2, epoch,
                                      draws)
        if self._grad is None:
            self._grad = torch.empty(self.engine.head_floats, dtype=torch.float32,
                                     device=imgs.device)
        grad = self.engine.head_backward(dkp, self._grad)
        scale = allreduce_head_grad(grad, self.group)   # RCCL over xGMI, 2.5 MB
        if update:
            self.engine.sgd_step(grad, self.lr * scale)
        return out, grad


class DescriptorLossGrad:
    """Descriptor-training loss (configs/train_desc.yaml) with its gradient:
    Preprocess_Line2Window (losses/preprocess.py:27-121) + EpipolarLoss_full
    (losses/epipolarloss.py:38-101) forward, then dL/d local_map for both
    images (what ``total_loss.backward()`` sends into the backbone at
    managers/trainer.py:331).  Three HIP calls: ``posfeat_line2window``,
    ``posfeat_epipolar_loss``, ``posfeat_line2window_backward``.

    ``__call__(x1, x2, F1, F2, hw1, hw2, epoch, draws=None)`` with x1/x2 the NHWC
    local maps ([b, h, w, >=128], channel stride = last dim) returns
    (out[7] = loss, loss_g1, loss_w1, loss_g2, loss_w2, percent_g, percent_w;
    dx1, dx2 NHWC [b, h, w, 128]; the processed dict's tensors)."""

    def __init__(self, pre_cfg, epi_cfg):
        from .losses.preprocess import Preprocess_Line2Window
        Preprocess_Line2Window(pre_cfg)            # validates the configuration
        if epi_cfg.get("weight_grid", 0) != 0 or not epi_cfg.get("use_std_as_weight", True):
            raise NotImplementedError("posfeat_amd implements the configs/train_desc.yaml "
                                      "EpipolarLoss_full (weight_grid 0, std weights)")
        self.pre = pre_cfg
        self.epi = epi_cfg
        self.grid = int(pre_cfg["kps_generator_config"]["grid_size"])
        self.line_step = int(pre_cfg.get("line_search_config", {}).get("line_step", 100))
        self._ws = {}

    def _buf(self, key, nbytes, dev):
        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
            self._ws[key] = t
        return t

    def __call__(self, x1, x2, F1, F2, hw1, hw2, epoch=1, draws=None):
        import ctypes
        b, h1, w1, cs1 = x1.shape
        _, h2, w2, cs2 = x2.shape
        (H1, W1), (H2, W2) = hw1, hw2
        dev = x1.device
        _lib.require_device(x1)
        g = self.grid
        n1, n2 = (H1 // g) * (W1 // g), (H2 // g) * (W2 // g)
        T = float(min(self.pre["temperature_base"] + epoch, self.pre["temperature_max"]))
        win = float(self.pre["window_size"])
        if draws is None:
            sel1 = torch.randint(0, g * g, (b, n1), device=dev, dtype=torch.int32)
            sel2 = torch.randint(0, g * g, (b, n2), device=dev, dtype=torch.int32)
            rand1 = torch.rand(b, n1, 2, device=dev)
            rand2 = torch.rand(b, n2, 2, device=dev)
        else:
            sel1, sel2, rand1, rand2 = [d.to(dev).contiguous() for d in draws]
            sel1, sel2 = sel1.reshape(b, n1).int(), sel2.reshape(b, n2).int()
        F1 = F1.to(dev).float().contiguous()
        F2 = F2.to(dev).float().contiguous()
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        res = {"coord1": f(b, n1, 2), "coord2": f(b, n2, 2), "g1": f(b, n1, 2), "g2": f(b, n2, 2),
               "g1_std": f(b, n1), "g2_std": f(b, n2), "l1_exp_n": f(b, n1, 2),
               "l2_exp_n": f(b, n2, 2), "l1_org_n": f(b, n1, 2), "l2_org_n": f(b, n2, 2),
               "valid1": torch.empty(b, n1, dtype=torch.uint8, device=dev),
               "valid2": torch.empty(b, n2, dtype=torch.uint8, device=dev),
               "w1": f(b, n1, 2), "w2": f(b, n2, 2), "w1_std": f(b, n1), "w2_std": f(b, n2)}
        o = _lib.L2WOut(**{k: v.data_ptr() for k, v in res.items()})
        L = lib()
        need = L.posfeat_line2window_workspace(b, H1, W1, H2, W2, g)
        fws = self._buf("fwd", need, dev)
        check(L.posfeat_line2window(ptr(x1), cs1, ptr(x2), cs2, b, H1, W1, H2, W2, ptr(F1),
                                    ptr(F2), ptr(sel1), ptr(sel2), ptr(rand1), ptr(rand2), T, g,
                                    win, self.line_step, ctypes.byref(o), ptr(fws), need,
                                    stream_ptr()))
        out = torch.empty(7, device=dev)
        short = float(min(H1, W1))
        args = [res[k] for k in ("coord1", "coord2", "g1", "g2", "w1", "w2", "g1_std", "g2_std",
                                 "w1_std", "w2_std")]
        check(L.posfeat_epipolar_loss(b, n1, ptr(F1), ptr(F2), *[ptr(a) for a in args],
                                      ptr(res["valid1"]), ptr(res["valid2"]), short,
                                      float(self.epi["grid_cost_thr"]),
                                      float(self.epi["win_cost_thr"]),
                                      float(self.epi["weight_grid"]),
                                      float(self.epi["weight_window"]), ptr(out), stream_ptr()))
        dx1 = torch.empty(b, h1, w1, 128, device=dev)
        dx2 = torch.empty(b, h2, w2, 128, device=dev)
        bneed = L.posfeat_line2window_backward_workspace(b, H1, W1, H2, W2, g)
        bws = self._buf("bwd", bneed, dev)
        check(L.posfeat_line2window_backward(
            ptr(x1), cs1, ptr(x2), cs2, b, H1, W1, H2, W2, ptr(F1), ptr(F2), ctypes.byref(o),
            ptr(fws), T, g, win, short, float(self.epi["grid_cost_thr"]),
            float(self.epi["win_cost_thr"]), float(self.epi["weight_grid"]),
            float(self.epi["weight_window"]), ptr(dx1), 128, ptr(dx2), 128, ptr(bws), bneed,
            stream_ptr()))
        return out, dx1, dx2, res


class BackboneTrainer:
    """Descriptor-training step (config 3, configs/train_desc.yaml): ResUNet in
    train mode (BatchNorm batch statistics + running update), the
    Line2Window/EpipolarLoss_full gradient, the backbone backward and Adam --
    one inner iteration of managers/trainer.py:293-356 with
    ``optimal_modules: ['backbone']``.  ``sync_bn=True`` under a process
    group of world > 1: SyncBatchNorm statistics over the ranks (RCCL inside
    the forward/backward, parallel.SyncBNGroup), as the reference's DDP
    wrapping converts the backbone (PoSFeat_model.py:49).

    State on the device: the packed parameter blob, its gradient, Adam's two
    moments (same layout) and the running-statistics blob.  One activation
    workspace per image batch (im1 and im2 are separate backbone calls in
    PoSFeat.forward, PoSFeat_model.py:144-145, so each has its own BN batch
    statistics and the running stats are updated twice per step); one
    scratch workspace shared by both.

    The keypoint head is not run: its output feeds neither this loss nor any
    state."""

    def __init__(self, backbone_sd, batch, h, w, device="cuda", lr=1e-4, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.0, momentum=0.1, group=None, sync_bn=False):
        import ctypes
        from . import weights
        _lib.require_device()
        # the training convs' tiles: exact tile-database entries only (the same
        # file on every rank -> the same tiles, engine.hip pf_conv_tuned_run)
        _load_tile_db()
        L = lib()
        self.table = _lib.bbtrain_table()
        params, stats = weights.pack_bbtrain(backbone_sd, self.table)
        dev = torch.device(device)
        self.device = dev
        self.params = torch.from_numpy(params).to(dev)
        self.stats = torch.from_numpy(stats).to(dev)
        self.grad = torch.zeros_like(self.params)   # conv_coarse never receives a gradient
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        nbt = [int(weights._np(v).reshape(-1)[0]) for k, v in backbone_sd.items()
               if k.endswith("num_batches_tracked")] if backbone_sd is not None else []
        self.num_batches_tracked = max(nbt) if nbt else 0
        self.adam_steps = 0
        self.lr, self.betas, self.eps, self.wd = float(lr), betas, float(eps), float(weight_decay)
        self.momentum = float(momentum)
        self.group = group
        self.batch, self.h, self.w = batch, h, w
        hnd = ctypes.c_void_p()
        check(L.posfeat_bbtrain_create(batch, h, w, ctypes.byref(hnd)))
        self._h = hnd
        na = L.posfeat_bbtrain_act_bytes(hnd)
        ns = L.posfeat_bbtrain_scratch_bytes(hnd)
        self.act = [torch.empty(na, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.scratch = torch.empty(ns, dtype=torch.uint8, device=dev)
        self._lm = [None, None]
        self._group = None
        if sync_bn and dist.is_available() and dist.is_initialized() \
                and dist.get_world_size(group) > 1:
            from .parallel import SyncBNGroup
            # SyncBatchNorm, PoSFeat_model.py:49 (same batch shape on every rank)
            self.set_group(SyncBNGroup(group, shape=(batch, h, w)))

    def set_group(self, group):
        """SyncBatchNorm: sum every BatchNorm's statistics over ``group``'s
        ranks (a parallel.SyncBNGroup, or a raw posfeat_group handle; None:
        per-rank statistics).  The group object must outlive its use here."""
        self._group = group
        h = getattr(group, "handle", group)
        check(lib().posfeat_bbtrain_set_group(self._h, h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().posfeat_bbtrain_destroy(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self._h = None

    def forward(self, img, slot):
        """Train-mode ResUNet on img [b,3,h,w] into workspace `slot` (0: im1,
        1: im2); returns the NHWC local map [b, h/4, w/4, 128] (a view into the
        workspace, valid until the next forward on that slot)."""
        import ctypes
        _lib.require_device(img)
        img = img.float().contiguous()
        out = ctypes.c_void_p()
        act = self.act[slot]
        check(lib().posfeat_bbtrain_forward(self._h, ptr(self.params), ptr(self.stats),
                                            self.momentum, ptr(img), ptr(act), ptr(self.scratch),
                                            ctypes.byref(out), stream_ptr()))
        self.num_batches_tracked += 1
        off = out.value - act.data_ptr()
        n = self.batch * (self.h // 4) * (self.w // 4) * 128
        lm = act[off:off + 4 * n].view(torch.float32).view(self.batch, self.h // 4, self.w // 4, 128)
        self._lm[slot] = lm
        return lm

    def backward(self, dlocal_map, slot, accumulate):
        """dL/d(local map of `slot`) (NHWC, last dim = pixel stride >= 128) ->
        grad (+)= dL/d params."""
        d = dlocal_map.float()
        if d.stride(-1) != 1 or d.stride(-2) != d.shape[-1]:
            d = d.contiguous()
        check(lib().posfeat_bbtrain_backward(self._h, ptr(self.params), ptr(self.act[slot]), ptr(d),
                                             d.shape[-1], ptr(self.grad), 1 if accumulate else 0,
                                             ptr(self.scratch), stream_ptr()))

    def adam_step(self, grad_scale=1.0):
        self.adam_steps += 1
        check(lib().posfeat_adam(ptr(self.params), ptr(self.grad), ptr(self.exp_avg),
                                 ptr(self.exp_avg_sq), self.params.numel(), self.lr,
                                 float(self.betas[0]), float(self.betas[1]), self.eps, self.wd,
                                 self.adam_steps, float(grad_scale), stream_ptr()))

    def step(self, im1, im2, F1, F2, loss, epoch=1, draws=None, update=True):
        """One training iteration: forward(im1), forward(im2), the loss and
        its map gradients (``loss``: a DescriptorLossGrad), backward of both
        batches into one gradient, RCCL all-reduce (world > 1), Adam.
        Returns (out[7], processed dict) as DescriptorLossGrad does."""
        x1 = self.forward(im1, 0)
        x2 = self.forward(im2, 1)
        hw = (int(im1.shape[2]), int(im1.shape[3]))
        out, dx1, dx2, res = loss(x1, x2, F1, F2, hw, (int(im2.shape[2]), int(im2.shape[3])),
                                  epoch=epoch, draws=draws)
        self.backward(dx1, 0, accumulate=False)
        self.backward(dx2, 1, accumulate=True)
        scale = allreduce_head_grad(self.grad, self.group)
        if update:
            self.adam_step(scale)
        return out, res

    def set_timing(self, enable):
        check(lib().posfeat_bbtrain_set_timing(self._h, 1 if enable else 0))

    def timing(self, prefix):
        import ctypes
        ms, fl, n = ctypes.c_double(), ctypes.c_double(), c_int()
        check(lib().posfeat_bbtrain_timing(self._h, prefix.encode(), ctypes.byref(ms),
                                           ctypes.byref(fl), ctypes.byref(n)))
        return ms.value, fl.value, n.value

    def timing_events(self, arith=False):
        """[(label, ms, flops)] of every timed launch of the last timed step
        (host-synchronises); ``arith=True`` appends the arithmetic mask of the
        label's MFMA launches (1 fp32 MFMA, 2 bf16x6, 3 both, 0 none)."""
        import ctypes
        out, i = [], 0
        lab, ms, fl = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_double()
        while lib().posfeat_bbtrain_timing_event(self._h, i, ctypes.byref(lab), ctypes.byref(ms),
                                                 ctypes.byref(fl)) == 0:
            ev = (lab.value.decode(), ms.value, fl.value)
            if arith:
                ev += (int(lib().posfeat_bbtrain_timing_event_arith(self._h, i)),)
            out.append(ev)
            i += 1
        return out

    def state_dict(self):
        """backbone.pth contents (reference key order, PoSFeat_model.py:74-81)."""
        from . import weights
        return weights.unpack_bbtrain(self.params.cpu().numpy(), self.table,
                                      self.stats.cpu().numpy(), self.num_batches_tracked)

    def grad_dict(self):
        from . import weights
        return weights.unpack_bbtrain(self.grad.cpu().numpy(), self.table)
