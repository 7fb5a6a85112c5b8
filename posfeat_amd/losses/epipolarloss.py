"""EpipolarLoss_full drop-in (reference: losses/epipolarloss.py:7-101).

``forward(inputs, outputs, processed) -> (loss, components)`` computed by one
HIP workgroup (posfeat_epipolar_loss).  When Preprocess_Line2Window ran on
local maps that require grad (``processed['_l2w']``), the loss is
differentiable: its backward is ``posfeat_line2window_backward`` (the fused
gradient of this loss through the window/grid expectations and their
softmax statistics into both NHWC local maps), laid back out as NCHW.
"""
import ctypes

import torch
import torch.nn as nn

from .. import ops
from .._lib import check, lib, ptr, stream_ptr


class EpipolarLoss_full(nn.Module):
    def __init__(self, configs, device=None):
        super().__init__()
        self.__lossname__ = "EpipolarLoss_fullinfo"
        self.config = configs
        self.w_g = self.config["weight_grid"]
        self.w_w = self.config["weight_window"]
        if not self.config.get("use_std_as_weight", True):
            raise NotImplementedError("use_std_as_weight=False is not implemented")

    def forward(self, inputs, outputs, processed):
        p = processed
        b, n = p["coord1"].shape[:2]
        if p["coord2"].shape[1] != n:
            raise NotImplementedError("both images must have the same grid size")
        dev = p["coord1"].device
        F1 = inputs["F1"].to(dev).float().contiguous()
        F2 = inputs["F2"].to(dev).float().contiguous()
        short = float(min(inputs["im1"].size()[2:]))
        v1 = p["valid_epi1"].to(torch.uint8).contiguous()
        v2 = p["valid_epi2"].to(torch.uint8).contiguous()
        out = torch.empty(7, device=dev)
        c = lambda k: p[k].float().contiguous()  # noqa: E731
        args = [c("coord1"), c("coord2"), c("feat1g_corloc"), c("feat2g_corloc"),
                c("feat1w_corloc"), c("feat2w_corloc"), c("feat1g_std"), c("feat2g_std"),
                c("feat1w_std"), c("feat2w_std")]
        check(lib().posfeat_epipolar_loss(b, n, ptr(F1), ptr(F2), *[ptr(a) for a in args],
                                          ptr(v1), ptr(v2), short,
                                          float(self.config["grid_cost_thr"]),
                                          float(self.config["win_cost_thr"]), float(self.w_g),
                                          float(self.w_w), ptr(out), stream_ptr()))
        loss = out[0]
        st = p.get("_l2w")
        if st is not None and torch.is_grad_enabled():
            loss = _EpipolarFn.apply(st["xf1"], st["xf2"], out[0], st, short, self.config)
        comp = {"loss_g1": out[1], "loss_w1": out[2], "loss_g2": out[3], "loss_w2": out[4],
                "percent_g": out[5], "percent_w": out[6]}
        return loss, comp


class _EpipolarFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xf1, xf2, loss, st, short, cfg):
        ctx.st, ctx.short, ctx.cfg = st, short, cfg
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        st, cfg = ctx.st, ctx.cfg
        b = st["b"]
        H1, W1, H2, W2 = st["hw"]
        x1, x2 = st["x1"], st["x2"]
        dev = x1.device
        L = lib()
        dx1 = torch.empty(b, x1.shape[1], x1.shape[2], 128, device=dev)
        dx2 = torch.empty(b, x2.shape[1], x2.shape[2], 128, device=dev)
        need = L.posfeat_line2window_backward_workspace(b, H1, W1, H2, W2, st["g"])
        bws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        check(L.posfeat_line2window_backward(
            ptr(x1), x1.shape[-1], ptr(x2), x2.shape[-1], b, H1, W1, H2, W2, ptr(st["F1"]),
            ptr(st["F2"]), ctypes.byref(st["o"]), ptr(st["ws"]), st["T"], st["g"], st["win"],
            float(ctx.short), float(cfg["grid_cost_thr"]), float(cfg["win_cost_thr"]),
            float(cfg["weight_grid"]), float(cfg["weight_window"]), ptr(dx1), 128, ptr(dx2), 128,
            ptr(bws), need, stream_ptr()))
        d1 = ops.nhwc_to_nchw(dx1) * g if st["xf1"].requires_grad else None
        d2 = ops.nhwc_to_nchw(dx2) * g if st["xf2"].requires_grad else None
        return d1, d2, None, None, None, None
