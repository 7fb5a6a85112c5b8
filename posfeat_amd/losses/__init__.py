"""Drop-in for the reference's ``losses`` package: ``preprocess_utils`` (the
extraction-path detector / sampler).  The training-side correlation modules
(Preprocess_Line2Window, EpipolarLoss_full, DiskLoss) are SURVEY §8 rows
a9-a11 and land in later rounds."""
from . import preprocess_utils  # noqa: F401
