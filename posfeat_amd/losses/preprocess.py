"""Preprocess_Line2Window drop-in (reference: losses/preprocess.py:10-129).

Same constructor ``(configs, device=None)`` and ``forward(inputs, outputs)``
returning the reference's dict; the whole forward runs in the HIP path
``posfeat_line2window`` (grid-point descriptors, MFMA cos-sim, row/column
softmax expectations, epipolar line search, window expectation).  Random
draws (the per-cell Categorical sample and the loc_rand jitter) are taken from
torch's device generator, or passed explicitly (``draws=``) for parity tests.

Autograd: when a local map requires grad (descriptor training), the forward
state (NHWC maps, draws, the kernel's workspace) is kept in
``processed['_l2w']`` and EpipolarLoss_full's differentiable loss runs
``posfeat_line2window_backward`` for dL/d local maps (the gradient the
reference's ``total_loss.backward()`` sends through these processed tensors).
Only the configuration of configs/train_desc.yaml is implemented; other
options raise NotImplementedError.
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib, ops
from .._lib import check, lib, ptr, stream_ptr


class Preprocess_Line2Window(nn.Module):
    def __init__(self, configs, device=None, vis=False):
        super().__init__()
        self.__lossname__ = "Preprocess_Line2Window"
        self.config = configs
        kg = self.config["kps_generator_config"]
        ls = self.config.get("line_search_config", {})
        if (self.config["kps_generator"] != "generate_kpts_regular_grid_random"
                or kg.get("map_init", "identity") != "identity"
                or kg.get("random_select", "random") != "random"
                or self.config.get("use_nn_grid", False)
                or not self.config.get("use_line_search", True)
                or not ls.get("use_nn", True) or not ls.get("loc_rand", True)
                or self.config.get("loss_distance", "cos") != "cos"):
            raise NotImplementedError("posfeat_amd implements the configs/train_desc.yaml "
                                      "Preprocess_Line2Window configuration")
        self.grid = int(kg["grid_size"])
        self.keep_spatial = bool(kg.get("keep_spatial", True))
        self.line_step = int(ls.get("line_step", 100))
        self.t_base = self.config["temperature_base"]
        self.t_max = self.config["temperature_max"]
        if device is not None:
            self.device = device

    def name(self):
        return self.__lossname__

    def forward(self, inputs, outputs, draws=None):
        xf1, xf2 = outputs["preds1"]["local_map"], outputs["preds2"]["local_map"]
        h1i, w1i = inputs["im1"].size()[2:]
        h2i, w2i = inputs["im2"].size()[2:]
        b = xf1.shape[0]
        T = float(min(self.t_base + outputs["epoch"], self.t_max))
        g = self.grid
        n1 = (h1i // g) * (w1i // g)
        n2 = (h2i // g) * (w2i // g)
        dev = xf1.device
        _lib.require_device(xf1)
        if draws is None:
            sel1 = torch.randint(0, g * g, (b, n1), device=dev, dtype=torch.int32)
            sel2 = torch.randint(0, g * g, (b, n2), device=dev, dtype=torch.int32)
            rand1 = torch.rand(b, n1, 2, device=dev)
            rand2 = torch.rand(b, n2, 2, device=dev)
        else:
            sel1, sel2, rand1, rand2 = [d.to(dev).contiguous() for d in draws]
            sel1, sel2 = sel1.reshape(b, n1).int(), sel2.reshape(b, n2).int()
        nh1 = getattr(outputs["preds1"], "local_map_nhwc", None)
        nh2 = getattr(outputs["preds2"], "local_map_nhwc", None)
        x1 = nh1 if nh1 is not None else ops.nchw_to_nhwc(xf1.detach().float().contiguous())
        x2 = nh2 if nh2 is not None else ops.nchw_to_nhwc(xf2.detach().float().contiguous())
        F1 = inputs["F1"].to(dev).float().contiguous()
        F2 = inputs["F2"].to(dev).float().contiguous()
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        res = {"coord1": f(b, n1, 2), "coord2": f(b, n2, 2), "g1": f(b, n1, 2), "g2": f(b, n2, 2),
               "g1_std": f(b, n1), "g2_std": f(b, n2), "l1_exp_n": f(b, n1, 2),
               "l2_exp_n": f(b, n2, 2), "l1_org_n": f(b, n1, 2), "l2_org_n": f(b, n2, 2),
               "valid1": torch.empty(b, n1, dtype=torch.uint8, device=dev),
               "valid2": torch.empty(b, n2, dtype=torch.uint8, device=dev),
               "w1": f(b, n1, 2), "w2": f(b, n2, 2), "w1_std": f(b, n1), "w2_std": f(b, n2)}
        o = _lib.L2WOut(**{k: v.data_ptr() for k, v in res.items()})
        need = lib().posfeat_line2window_workspace(b, h1i, w1i, h2i, w2i, g)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        check(lib().posfeat_line2window(ptr(x1), x1.shape[-1], ptr(x2), x2.shape[-1], b, h1i,
                                        w1i, h2i, w2i, ptr(F1), ptr(F2), ptr(sel1), ptr(sel2),
                                        ptr(rand1), ptr(rand2), T, g,
                                        float(self.config["window_size"]), self.line_step,
                                        ctypes.byref(o), ptr(ws), need, stream_ptr()))
        self.last_raw = res   # the kernel's raw outputs (line centres etc.), for diagnostics
        c1 = torch.tensor([(w2i - 1) / 2.0, (h2i - 1) / 2.0], device=dev)
        grad = torch.is_grad_enabled() and (xf1.requires_grad or xf2.requires_grad)
        state = None
        if grad:   # everything posfeat_line2window_backward reads, kept alive
            state = {"xf1": xf1, "xf2": xf2, "x1": x1, "x2": x2, "F1": F1, "F2": F2, "o": o,
                     "res": res, "ws": ws, "T": T, "g": g, "win": float(self.config["window_size"]),
                     "hw": (h1i, w1i, h2i, w2i), "b": b}
        return {
            "_l2w": state,
            "coord1": res["coord1"], "coord2": res["coord2"],
            "feat1g_corloc": res["g1"], "feat2g_corloc": res["g2"],
            "feat1w_corloc": res["w1"], "feat2w_corloc": res["w2"],
            "feat1c_corloc_org": res["l1_org_n"] * c1 + c1,
            "feat2c_corloc_org": res["l2_org_n"],  # sic (preprocess.py:116)
            "feat1g_std": res["g1_std"], "feat2g_std": res["g2_std"],
            "feat1w_std": res["w1_std"], "feat2w_std": res["w2_std"],
            "temperature": T,
            "valid_epi1": res["valid1"].bool(), "valid_epi2": res["valid2"].bool(),
        }


class Preprocess_Skip(nn.Module):
    def __init__(self, **kargs):
        super().__init__()
        self.__lossname__ = "Preprocess_Skip"

    def forward(self, inputs, outputs):
        return None
