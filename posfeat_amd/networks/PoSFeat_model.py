"""PoSFeat drop-in (reference: networks/PoSFeat_model.py:15-147).

Keeps the constructor ``PoSFeat(configs, device, no_cuda=None)``, the
attributes (``backbone``, ``localheader``, ``parameters``, ``modules``) and the
methods ``set_parallel``, ``load_checkpoint``, ``save_checkpoint``,
``set_train``, ``set_eval``, ``extract`` and ``forward``.

``extract`` runs the whole ResUNet + KeypointDet forward as one call into the
HIP engine (posfeat_model_extract) with BN folded into packed weights that
are rebuilt whenever the parameters change.  As in the reference the modules
live on ``device``.

``forward`` under autograd follows the reference Trainer
(managers/trainer.py:296-331; posfeat_amd.autograd):
* ``localheader`` in train mode (configs/train_kp.yaml): im1 and im2 run as one
  batch through an ExtractionEngine(train=True) (instance norm is per image
  and the frozen backbone uses eval BatchNorm, so batching is exact); the
  ``local_point`` maps are differentiable w.r.t. ``localheader``'s parameters.
* ``backbone`` in train mode (configs/train_desc.yaml): im1 and im2 run as two
  train-mode ResUNet calls (own BatchNorm batch statistics each, running
  statistics updated twice, as PoSFeat_model.py:144-145 does); ``local_map``
  is differentiable w.r.t. ``backbone``'s parameters; after ``set_parallel``
  its BatchNorms are SyncBatchNorms (statistics summed over the ranks by RCCL
  inside the forward/backward) and the gradients are averaged over the ranks,
  as the reference's SyncBN + DDP wrapping does.  The keypoint head's
  output feeds neither the descriptor loss nor any state, so ``local_point``,
  ``global_map`` and ``global_feat`` are None there.
Differences from the reference are loud, never silent: CPU devices raise.
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
        self.backbone = ResUNet(**self.config["backbone_config"]).to(self.device)
        self.parameters += list(self.backbone.parameters())
        message = "backbone: {}\n".format(self.config["backbone"])
        if "localheader" in list(self.config.keys()) and self.config["localheader"] != "None":
            if self.config["localheader"] != "KeypointDet":
                raise NotImplementedError("localheader must be 'KeypointDet'")
            self.localheader = KeypointDet(**self.config["localheader_config"]).to(self.device)
            message += "localheader: {}\n".format(self.config["localheader"])
        else:
            # reference default: KeypointDet(in_channels=out_channels[0], out_channels=2)
            raise NotImplementedError("the 2-channel default KeypointDet head is not implemented")
        self.parameters += list(self.localheader.parameters())
        self.modules = ["localheader", "backbone"]
        self._engine = None
        self._engine_key = None
        self._parallel = False
        self._head_train = None      # (backbone key, ExtractionEngine(train=True), HeadBinding)
        self._bb_train = {}          # (b, h, w) -> BackboneBinding
        print(message)

    # ------------------------------------------------------------------ engine
    def _param_key(self):
        return tuple(p._version for p in self.backbone.state_dict(keep_vars=True).values()) + \
            tuple(p._version for p in self.localheader.state_dict(keep_vars=True).values())

    def engine(self):
        from ..engine import ExtractionEngine
        weights.materialize_seed(self.backbone)   # built inside weights.deferred_seed()
        weights.materialize_seed(self.localheader)
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
        independently (no per-forward buffer broadcast, no grad all-reduce).
        For training through ``forward`` (posfeat_amd.autograd) the gradients
        are then averaged over the ranks (one all-reduce of the packed
        gradient per module and step) and the train-mode backbone uses
        SyncBatchNorm statistics (parallel.SyncBNGroup)."""
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
                weights.materialize_seed(getattr(self, name))
                continue
            print("load {} from checkpoint".format(name))
            getattr(self, name).load_state_dict(sd)
            getattr(self, name)._seed_pending = None   # every tensor replaced (strict load)
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

    # ------------------------------------------------------------------ training
    def _bb_key(self):
        return tuple(p._version for p in self.backbone.state_dict(keep_vars=True).values())

    def _head_binding(self):
        from ..autograd import HeadBinding
        from ..engine import ExtractionEngine
        key = self._bb_key()
        if self._head_train is None or self._head_train[0] != key:
            eng = ExtractionEngine(self.backbone.state_dict(), self.localheader.state_dict(),
                                   device=self.device, train=True)
            self._head_train = (key, eng, HeadBinding(eng, self.localheader))
        binding = self._head_train[2]
        binding.parallel = self._parallel
        binding.sync()
        return binding

    def _forward_head_train(self, im1, im2):
        from ..autograd import HeadFn
        binding = self._head_binding()
        b = im1.shape[0]
        imgs = torch.cat([im1, im2], 0).float().contiguous()
        res = binding.engine.run(imgs, outputs=("local_map", "global_map", "global_feat"))
        binding.token += 1
        lp = HeadFn.apply(res["local_point"], binding, binding.token, *binding.params)
        preds = []
        for sl in (slice(0, b), slice(b, 2 * b)):
            g = res["global_map"][sl]
            o = ExtractOutputs(local_map=res["local_map"][sl], global_map=g,
                               global_feat=res["global_feat"][sl], local_point=lp[sl],
                               local_thr=torch.zeros_like(lp[sl]),
                               global_point=torch.ones(g.shape[0], 1, g.shape[2], g.shape[3],
                                                       device=g.device))
            o.local_map_nhwc = res["_local_map_nhwc"][sl]
            preds.append(o)
        return preds

    def _syncbn_group(self):
        if getattr(self, "_sbn", None) is None:
            from ..parallel import SyncBNGroup
            self._sbn = SyncBNGroup()
        return self._sbn

    def _forward_backbone_train(self, im1, im2):
        from .. import ops
        from ..autograd import BackboneBinding, BackboneFn
        preds = []
        for slot, im in enumerate((im1, im2)):
            b, _, h, w = im.shape
            binding = self._bb_train.get((b, h, w))
            if binding is None:
                binding = self._bb_train[(b, h, w)] = BackboneBinding(self.backbone, b, h, w,
                                                                      self.device)
            binding.parallel = self._parallel
            if self._parallel and binding.trainer._group is None:
                binding.trainer.set_group(self._syncbn_group())   # SyncBatchNorm
            lm_nhwc = binding.forward(im.float().contiguous(), slot)
            lm = BackboneFn.apply(ops.nhwc_to_nchw(lm_nhwc), binding, slot,
                                  binding.tokens[slot], *binding.params)
            o = ExtractOutputs(local_map=lm, global_map=None, global_feat=None, local_point=None,
                               local_thr=None, global_point=None)
            o.local_map_nhwc = lm_nhwc
            preds.append(o)
        return preds

    def forward(self, inputs):
        for key, val in inputs.items():
            if key in self.no_cuda:
                continue
            inputs[key] = val.to(self.device)
        if torch.is_grad_enabled() and self.backbone.training:
            preds1, preds2 = self._forward_backbone_train(inputs["im1"], inputs["im2"])
            return {"preds1": preds1, "preds2": preds2}
        if torch.is_grad_enabled() and self.localheader.training:
            preds1, preds2 = self._forward_head_train(inputs["im1"], inputs["im2"])
            return {"preds1": preds1, "preds2": preds2}
        preds1 = self.extract(inputs["im1"], 1)
        preds1.local_map_nhwc = None  # workspace is reused by the next extract
        preds2 = self.extract(inputs["im2"], 2)
        return {"preds1": preds1, "preds2": preds2}

    __call__ = forward
