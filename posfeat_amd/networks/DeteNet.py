"""KeypointDet drop-in (reference: networks/DeteNet.py:9-121).

Same constructor and 9-key state dict.  The configuration used by every
reference config (in_channels=192, out_channels=1, prior='identity',
act='Softplus') runs in the HIP engine: fused with the backbone via
PoSFeat.extract, or standalone here (``forward([x, img])``, the engine's
head-only mode); other priors/activations raise NotImplementedError.
"""
import torch.nn as nn

from .. import weights
from ._params import build_param_tree


class KeypointDet(nn.Module):
    def __init__(self, in_channels, out_channels=1, prior="SSIM", act="Sigmoid"):
        super().__init__()
        if in_channels != 192 or out_channels != 1 or prior != "identity" or act != "Softplus":
            raise NotImplementedError(
                "posfeat_amd implements KeypointDet(in_channels=192, out_channels=1, "
                "prior='identity', act='Softplus') -- configs/train_desc.yaml:24-28")
        build_param_tree(self, weights.head_param_shapes(in_channels, out_channels))
        weights.seed_module(self, "localheader")

    def forward(self, fine_maps):
        """fine_maps = [x, img]: x = cat[local_map, local_map_small] [b,192,h/4,w/4],
        img [b,3,h,w] -> score map [b,1,h,w] (DeteNet.py:102-121; the identity
        prior multiplies by exactly 1).  Eval only: gradients come from the
        engine's head backward (training.KeypointTrainStep)."""
        from ..engine import keypointdet_forward
        x, img = fine_maps[0], fine_maps[1]
        return keypointdet_forward(self, x, img)
