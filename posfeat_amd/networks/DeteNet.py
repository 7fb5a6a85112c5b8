"""KeypointDet drop-in (reference: networks/DeteNet.py:9-121).

Same constructor and 9-key state dict.  The configuration used by every
reference config (in_channels=192, out_channels=1, prior='identity',
act='Softplus') runs inside the fused HIP engine via PoSFeat.extract; other
priors/activations raise NotImplementedError.
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
        _, hd = weights.seeded_state_dicts(0)
        self.load_state_dict(hd)

    def forward(self, fine_maps):
        raise NotImplementedError(
            "KeypointDet runs fused with the backbone in the HIP engine: call "
            "PoSFeat.extract(img) (networks/PoSFeat_model.py:91-134)")
