"""posfeat_amd -- MI355X-native PoSFeat extraction + correlation hot path.

Host side mirrors the reference's Python surfaces (``networks.PoSFeat``,
``losses.preprocess_utils``, ``managers.extractor.Extractor``); all device
arithmetic runs in hand-written gfx950 HIP kernels in ``libposfeat_hip.so``
reached through a C ABI (``include/posfeat_hip.h``).  Importing this package
does not load the library; the first op call does, and fails loudly if it is
missing.
"""
__version__ = "0.1.0"
