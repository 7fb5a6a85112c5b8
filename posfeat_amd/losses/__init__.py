"""Drop-in for the reference's ``losses`` package (losses/__init__.py):
``preprocess_utils`` (extraction detector / sampler), ``Preprocess_Line2Window``
and ``Preprocess_Skip`` (preprocess.py), ``EpipolarLoss_full``
(epipolarloss.py) and ``DiskLoss`` (kploss.py) on the HIP path; the losses
are differentiable (torch.autograd.Function over the fused gradient kernels)
when their input maps require grad."""
from . import preprocess_utils  # noqa: F401
from .preprocess import Preprocess_Line2Window, Preprocess_Skip  # noqa: F401
from .epipolarloss import EpipolarLoss_full  # noqa: F401
from .kploss import DiskLoss  # noqa: F401
