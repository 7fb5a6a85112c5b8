"""Drop-in for the reference's ``networks`` package (networks/__init__.py):
``ResUNet``, ``KeypointDet`` and ``PoSFeat`` with the same constructor
arguments, state-dict layouts and methods; arithmetic runs in the HIP engine."""
from .DescNet import ResUNet
from .DeteNet import KeypointDet
from .PoSFeat_model import PoSFeat

__all__ = ["ResUNet", "KeypointDet", "PoSFeat"]
