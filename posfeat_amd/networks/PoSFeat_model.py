"""PoSFeat drop-in (reference: networks/PoSFeat_model.py:15-147).

Keeps the constructor ``PoSFeat(configs, device, no_cuda=None)``, the
attributes (``backbone``, ``localheader``, ``parameters``, ``modules``) and the
methods ``set_parallel``, ``load_checkpoint``, ``save_checkpoint``,
``set_train``, ``set_eval``, ``extract`` and ``forward``.

``extract`` runs the whole ResUNet + KeypointDet forward as one call into the
HIP engine (posfeat_model_extract) with BN folded into packed weights that
are rebuilt whenever the parameters change.  Differences from the reference
are loud, never silent: training-mode extraction (batch-stat BN) and CPU
devices raise.
"""
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F  # noqa: F401  (API parity with the reference module)

from .. import weights
from .DescNet import ResUNet
from .DeteNet import KeypointDet


class ExtractOutputs(dict):
    """The reference's output dict (PoSFeat_model.py:119-126) plus an
    attribute ``local_map_nhwc``: the engine's NHWC copy of local_map (a view
    into the engine workspace, valid until the next extract of that shape),
    used by the fused Extractor.process path for coalesced sampling."""
    local_map_nhwc = None


class PoSFeat:
    def __init__(self, configs, device, no_cuda=None):
        self.config = configs
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        self.no_cuda = no_cuda if no_cuda is not None else []
        self.align_local_grad = self.config["align_local_grad"]
        self.local_input_elements = self.config["local_input_elements"]
        self.local_with_img = self.config["local_with_img"]
        if list(self.local_input_elements) != ["local_map", "local_map_small"] \
                or not self.local_with_img:
            raise NotImplementedError(
                "posfeat_amd implements local_input_elements=['local_map','local_map_small'], "
                "local_with_img=True (configs/train_desc.yaml:29-31)")
        self.parameters = []
        if self.config["backbone"] != "ResUNet":
            raise NotImplementedError("backbone must be 'ResUNet'")
        self.backbone = ResUNet(**self.config["backbone_config"])
        self.parameters += list(self.backbone.parameters())
        message = "backbone: {}\n".format(self.config["backbone"])
        if "localheader" in list(self.config.keys()) and self.config["localheader"] != "None":
            if self.config["localheader"] != "KeypointDet":
                raise NotImplementedError("localheader must be 'KeypointDet'")
            self.localheader = KeypointDet(**self.config["localheader_config"])
            message += "localheader: {}\n".format(self.config["localheader"])
        else:
            # reference default: KeypointDet(in_channels=out_channels[0], out_channels=2)
            raise NotImplementedError("the 2-channel default KeypointDet head is not implemented")
        self.parameters += list(self.localheader.parameters())
        self.modules = ["localheader", "backbone"]
        self._engine = None
        self._engine_key = None
        self._parallel = False
        print(message)

    # ------------------------------------------------------------------ engine
    def _param_key(self):
        return tuple(p._version for p in self.backbone.state_dict(keep_vars=True).values()) + \
            tuple(p._version for p in self.localheader.state_dict(keep_vars=True).values())

    def engine(self):
        from ..engine import ExtractionEngine
        key = self._param_key()
        if self._engine is None or key != self._engine_key:
            self._engine = ExtractionEngine(self.backbone.state_dict(),
                                            self.localheader.state_dict(), device=self.device)
            self._engine_key = key
        return self._engine

    # ------------------------------------------------------------------ API
    def set_parallel(self, local_rank):
        """Reference: SyncBN + DDP wrappers (PoSFeat_model.py:48-55).  For
        extraction the only collective needed is making every rank hold rank
        0's weights: one RCCL broadcast per tensor; ranks then run
        independently (no per-forward buffer broadcast, no grad all-reduce)."""
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("set_parallel needs an initialised process group")
        from ..parallel import broadcast_weights
        broadcast_weights([self.backbone.state_dict(), self.localheader.state_dict()],
                          device=self.device)
        self._parallel = True
        self._engine = None

    def load_checkpoint(self, load_path):
        bb, hd = weights.load_checkpoint_dir(load_path)
        for name, sd in (("backbone", bb), ("localheader", hd)):
            if sd is None:
                print("{} does not exist, skipping load".format(name))
                continue
            print("load {} from checkpoint".format(name))
            getattr(self, name).load_state_dict(sd)
        self._engine = None

    def save_checkpoint(self, save_path):
        os.makedirs(str(save_path), exist_ok=True)
        for name in ("backbone", "localheader"):
            torch.save(getattr(self, name).state_dict(),
                       os.path.join(str(save_path), "{}.pth".format(name)))

    def set_train(self):
        self.backbone.train()
        self.localheader.train()

    def set_eval(self):
        self.backbone.eval()
        self.localheader.eval()

    def extract(self, tensor, postfix=""):
        if self.backbone.training:
            raise NotImplementedError(
                "train-mode (batch-statistics BN) extraction is not implemented; call set_eval()")
        if tensor.device.type != "cuda":
            tensor = tensor.to(self.device)
        out = self.engine().run(tensor.float(), outputs=("local_map", "global_map", "global_feat"))
        b, _, h, w = out["global_map"].shape
        g_map = torch.ones(b, 1, h, w, device=tensor.device, dtype=torch.float32)
        res = ExtractOutputs(
            local_map=out["local_map"], global_map=out["global_map"],
            global_feat=out["global_feat"], local_point=out["local_point"],
            local_thr=torch.zeros_like(out["local_point"]), global_point=g_map)
        res.local_map_nhwc = out["_local_map_nhwc"]
        return res

    def forward(self, inputs):
        for key, val in inputs.items():
            if key in self.no_cuda:
                continue
            inputs[key] = val.to(self.device)
        preds1 = self.extract(inputs["im1"], 1)
        preds1.local_map_nhwc = None  # workspace is reused by the next extract
        preds2 = self.extract(inputs["im2"], 2)
        return {"preds1": preds1, "preds2": preds2}

    __call__ = forward
