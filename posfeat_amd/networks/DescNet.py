"""ResUNet drop-in (reference: networks/DescNet.py:12-84).

Same constructor, same 300-key state dict (torchvision ResNet-50 encoder
through layer3 + conv_coarse/upconv3/iconv3/upconv2/iconv2/conv_fine).
``forward`` runs the HIP engine and returns the reference's dict
(global_map, local_map, local_map_small).  Only the configuration the
reference's configs use is implemented (encoder='resnet50', 128/128); other
encoders raise NotImplementedError instead of silently falling back.
"""
import torch.nn as nn

from .. import weights
from ._params import build_param_tree


class ResUNet(nn.Module):
    def __init__(self, encoder="resnet50", pretrained=True, coarse_out_ch=128, fine_out_ch=128):
        super().__init__()
        assert encoder in ["resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
                           "wide_resnet50_2"], "Incorrect encoder type"
        if encoder != "resnet50" or coarse_out_ch != 128 or fine_out_ch != 128:
            raise NotImplementedError(
                "posfeat_amd implements ResUNet(encoder='resnet50', coarse_out_ch=128, "
                "fine_out_ch=128) -- the configuration of configs/train_desc.yaml")
        # `pretrained` would download ImageNet weights in the reference; here the
        # parameters start from the seeded recipe and are replaced by
        # load_checkpoint / load_state_dict exactly as in the reference flow.
        build_param_tree(self, weights.backbone_param_shapes())
        weights.seed_module(self, "backbone")
        self.out_channels = [fine_out_ch, coarse_out_ch]
        self._runner = None

    def forward(self, x):
        from ..engine import backbone_forward
        return backbone_forward(self, x)
