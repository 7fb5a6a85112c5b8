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
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr
from .engine import ExtractionEngine
from .parallel import allreduce_head_grad

DISK_DEFAULTS = {"grid_size": 8, "loss_distance": "cos", "temperature_base": 60,
                 "temperature_max": 60, "epipolar_reward": "constant_reward",
                 "reward_config": {"reward_thr": 2, "rescale_thr": False}, "cor_detach": True,
                 "good_reward": 1, "bad_reward": -0.25, "kp_penalty": -0.001,
                 "match_grad": False}


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
