"""EpipolarLoss_full drop-in (reference: losses/epipolarloss.py:7-101).

``forward(inputs, outputs, processed) -> (loss, components)`` computed by one
HIP workgroup (posfeat_epipolar_loss).  Forward values only (no autograd yet).
"""
import torch
import torch.nn as nn

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

    @torch.no_grad()
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
        comp = {"loss_g1": out[1], "loss_w1": out[2], "loss_g2": out[3], "loss_w2": out[4],
                "percent_g": out[5], "percent_w": out[6]}
        return out[0], comp
