"""Drop-in for the reference's ``losses`` package (losses/__init__.py):
``preprocess_utils`` (extraction detector / sampler), ``Preprocess_Line2Window``
and ``Preprocess_Skip`` (preprocess.py), ``EpipolarLoss_full``
(epipolarloss.py) and ``DiskLoss`` (kploss.py) -- forward values on the HIP
path."""
from . import preprocess_utils  # noqa: F401
from .preprocess import Preprocess_Line2Window, Preprocess_Skip  # noqa: F401
from .epipolarloss import EpipolarLoss_full  # noqa: F401
from .kploss import DiskLoss  # noqa: F401
