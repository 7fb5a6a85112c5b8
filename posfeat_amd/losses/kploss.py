"""DiskLoss drop-in (reference: losses/kploss.py:7-197).

``DiskLoss(configs, device)`` with ``forward(inputs, outputs, processed)``
returning ``(loss, components)``; one HIP call (posfeat_disk_loss): per-cell
Categorical/Bernoulli sampling (Gumbel-max from device uniforms, or explicit
``draws=(prop1, prop2, acc1, acc2)`` for parity tests), descriptors at the
proposals, MFMA cos-sim, row/column log-sum-exp, and a fused reward x
probability reduction that never materialises the B x n x n probability
matrices.  Implemented for configs/train_kp.yaml (grid 8, constant_reward
without threshold rescaling).

Autograd: when a score map requires grad (the reference Trainer's
``total_loss.backward()``, managers/trainer.py:331), the loss comes from
``posfeat_disk_loss_grad`` -- the same values plus dL/d score maps in one call
-- wrapped in a ``torch.autograd.Function`` whose backward returns those maps
times the incoming gradient.  Descriptors receive no gradient: with
``cor_detach: True`` and ``match_grad: False`` (configs/train_kp.yaml) the
reference's loss does not differentiate through them (kploss.py:155-169), and
other settings raise.
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib, ops
from .._lib import check, lib, ptr, stream_ptr


class DiskLoss(nn.Module):
    def __init__(self, configs, device=None):
        super().__init__()
        self.__lossname__ = "DiskLoss"
        self.config = configs
        self.unfold_size = self.config["grid_size"]
        self.t_base = self.config["temperature_base"]
        self.t_max = self.config["temperature_max"]
        self.good_reward = self.config["good_reward"]
        self.bad_reward = self.config["bad_reward"]
        self.kp_penalty = self.config["kp_penalty"]
        rc = self.config.get("reward_config", {})
        if (self.unfold_size != 8 or self.config["epipolar_reward"] != "constant_reward"
                or rc.get("rescale_thr", False)
                or self.config.get("loss_distance", "cos") != "cos"):
            raise NotImplementedError("posfeat_amd implements the configs/train_kp.yaml DiskLoss")
        self.reward_thr = float(rc.get("reward_thr", 2))

    def forward(self, inputs, outputs, processed=None, draws=None):
        p1, p2 = outputs["preds1"], outputs["preds2"]
        kp1, kp2 = p1["local_point"], p2["local_point"]
        b, _, h, w = kp1.shape
        dev = kp1.device
        _lib.require_device(kp1)
        T = float(min(self.t_base + outputs["epoch"], self.t_max))
        n = (h // 8) * (w // 8)
        x1 = getattr(p1, "local_map_nhwc", None)
        x2 = getattr(p2, "local_map_nhwc", None)
        x1 = x1 if x1 is not None else ops.nchw_to_nhwc(p1["local_map"].float().contiguous())
        x2 = x2 if x2 is not None else ops.nchw_to_nhwc(p2["local_map"].float().contiguous())
        F1 = inputs["F1"].to(dev).float().contiguous()
        F2 = inputs["F2"].to(dev).float().contiguous()
        if draws is None:
            uni1 = torch.rand(b, n, 65, device=dev)
            uni2 = torch.rand(b, n, 65, device=dev)
            pr1 = pr2 = ac1 = ac2 = None
        else:
            pr1, pr2, ac1, ac2 = [d.to(dev).reshape(b, n).contiguous() for d in draws]
            pr1, pr2 = pr1.int(), pr2.int()
            ac1, ac2 = ac1.to(torch.uint8), ac2.to(torch.uint8)
            uni1 = uni2 = None
        out = torch.empty(4, device=dev)
        one = torch.ones((), device=dev)
        if torch.is_grad_enabled() and (kp1.requires_grad or kp2.requires_grad):
            if not self.config.get("cor_detach", True) or self.config.get("match_grad", False):
                raise NotImplementedError("DiskLoss gradients need cor_detach: True and "
                                          "match_grad: False (configs/train_kp.yaml)")
            k1 = kp1.detach().float().contiguous()
            k2 = kp2.detach().float().contiguous()
            d1, d2 = torch.empty_like(k1), torch.empty_like(k2)
            need = lib().posfeat_disk_loss_grad_workspace(b, h, w)
            ws = torch.empty(need, dtype=torch.uint8, device=dev)
            check(lib().posfeat_disk_loss_grad(
                ptr(k1), ptr(k2), ptr(x1), x1.shape[-1], ptr(x2), x2.shape[-1], b, h, w, ptr(F1),
                ptr(F2), ptr(pr1), ptr(pr2), ptr(ac1), ptr(ac2), ptr(uni1), ptr(uni2), T,
                self.reward_thr, float(self.good_reward), float(self.bad_reward),
                float(self.kp_penalty), ptr(out), ptr(d1), ptr(d2), ptr(ws), need, stream_ptr()))
            loss = _DiskLossFn.apply(kp1, kp2, out[0], d1, d2)
            comp = {"reinforce": out[1], "kp_penalty": out[2], "scale1": one, "scale2": one,
                    "n_kps": out[3], "temperature": torch.tensor(T, device=dev)}
            return loss, comp
        need = lib().posfeat_disk_loss_workspace(b, h, w)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        check(lib().posfeat_disk_loss(ptr(kp1.float().contiguous()), ptr(kp2.float().contiguous()),
                                      ptr(x1), x1.shape[-1], ptr(x2), x2.shape[-1], b, h, w,
                                      ptr(F1), ptr(F2), ptr(pr1), ptr(pr2), ptr(ac1), ptr(ac2),
                                      ptr(uni1), ptr(uni2), T, self.reward_thr,
                                      float(self.good_reward), float(self.bad_reward),
                                      float(self.kp_penalty), ptr(out), ptr(ws), need,
                                      stream_ptr()))
        comp = {"reinforce": out[1], "kp_penalty": out[2], "scale1": one, "scale2": one,
                "n_kps": out[3], "temperature": torch.tensor(T, device=dev)}
        return out[0], comp


class _DiskLossFn(torch.autograd.Function):
    """loss = out[0] of posfeat_disk_loss_grad; d loss / d kp = the kernel's maps."""

    @staticmethod
    def forward(ctx, kp1, kp2, loss, d1, d2):
        ctx.save_for_backward(d1, d2)
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        d1, d2 = ctx.saved_tensors
        return d1 * g, d2 * g, None, None, None
