"""Evaluation matchers on the GPU -- drop-ins with the
reference's names, arguments and return values:

  mnn_matcher(descriptors_a, descriptors_b)        losses/preprocess_utils.py:795-803,
                                                   evaluations/hpatches/evaluation.py:28-38
  mutual_nn_matcher(descriptors1, descriptors2)    evaluations/aachen/matchers.py:5-14,
                                                   ETH_local_feature/custom_matcher.py:5-14
  ratio_matcher(descriptors1, descriptors2, ratio=0.95)            aachen/matchers.py:17-44
  mutual_nn_ratio_matcher(descriptors1, descriptors2, ratio=0.95)  aachen/matchers.py:47-75

Each returns the int64 numpy array [n_matches, 2] of (index in 1, index in 2),
ascending in the first index.  One call = two launches of the fused
MFMA-similarity + top-2 kernel (match.hip; the n1 x n2 similarity matrix is
never written) and one selection kernel; the host reads the match count once
(the reference's ``.cpu().numpy()`` synchronises there too).  Tie rule: the
first (lowest) index wins an arg-max tie.  Descriptors must be L2-normalised
128-d float32 (what Extractor.save_desc writes); numpy inputs are uploaded to
the current device.  No CPU path.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr

_MODES = {"mnn": 0, "ratio": 1, "mnn_ratio": 2}


def _dev(x):
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    if x.device.type != "cuda":
        _lib.require_device()
        x = x.to(torch.device("cuda", torch.cuda.current_device()))
    return x.float().contiguous()


def _match(d1, d2, mode, ratio=0.95):
    d1, d2 = _dev(d1), _dev(d2)
    _lib.require_device(d1)
    if d1.dim() != 2 or d2.dim() != 2 or d1.shape[1] != d2.shape[1]:
        raise ValueError("descriptors must be [n1, d] and [n2, d]")
    n1, dim = d1.shape
    n2 = d2.shape[0]
    if mode != "mnn" and min(n1, n2) < 2:
        # the reference's torch.topk(sim, 2, dim=1) / topk(sim.t(), 2, dim=1)
        # (aachen/matchers.py:21, 29, 51, 59) raise here; a second-best
        # similarity of -inf would instead pass every row through the ratio test
        raise RuntimeError("ratio matchers need at least 2 descriptors on each side "
                           "(got %d and %d): selected index k out of range" % (n1, n2))
    if n1 == 0 or n2 == 0:
        return np.zeros((0, 2), dtype=np.int64)
    if dim != 128:
        raise NotImplementedError("the matcher kernel is built for 128-d descriptors")
    need = lib().posfeat_match_workspace(n1, n2)
    ws = torch.empty(need, dtype=torch.uint8, device=d1.device)
    out = torch.empty(n1, 2, dtype=torch.int32, device=d1.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=d1.device)
    check(lib().posfeat_match(ptr(d1), n1, ptr(d2), n2, dim, _MODES[mode], float(ratio),
                              ptr(out), ptr(cnt), ptr(ws), need, stream_ptr()))
    n = int(cnt.item())
    return out[:n].cpu().numpy().astype(np.int64)


def mnn_matcher(descriptors_a, descriptors_b):
    return _match(descriptors_a, descriptors_b, "mnn")


def mutual_nn_matcher(descriptors1, descriptors2, **args):
    return _match(descriptors1, descriptors2, "mnn")


def ratio_matcher(descriptors1, descriptors2, ratio=0.95):
    return _match(descriptors1, descriptors2, "ratio", ratio)


def mutual_nn_ratio_matcher(descriptors1, descriptors2, ratio=0.95):
    return _match(descriptors1, descriptors2, "mnn_ratio", ratio)
