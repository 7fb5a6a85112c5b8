"""Intrinsic fp32 noise of the reference backbone gradients (tests/golden/bb_grad.npz):
the oracle run in fp64 against the fp32 reference fixture, per tensor
max|g64 - g_ref| / max|g_ref|.  Sets the scale for the HIP path's tolerance."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from oracle.model_ref import resunet_forward  # noqa: E402
from posfeat_amd.weights import seeded_state_dicts  # noqa: E402
from test_bb_train import _inputs  # noqa: E402


def main():
    d, im1, im2, R1, R2 = _inputs()
    bb, _ = seeded_state_dicts(0)
    sd = {k: (v.clone().double() if v.is_floating_point() else v.clone()) for k, v in bb.items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items()
              if not ("running" in k or "num_batches" in k)}
    o1 = resunet_forward(sd, im1.double(), train=True)
    o2 = resunet_forward(sd, im2.double(), train=True)
    loss = (o1["local_map"] * R1.double()).sum() + (o2["local_map"] * R2.double()).sum()
    keys = [k for k in params if "stat_" + k in d.files]
    grads = torch.autograd.grad(loss, [params[k] for k in keys])
    res = []
    for k, g in zip(keys, grads):
        if k.endswith("conv.bias"):
            continue
        g = g.numpy()
        if "grad_" + k in d.files:
            ref = d["grad_" + k].astype(np.float64)
            gg = g.reshape(ref.shape)
        else:
            ref = d["val_" + k].astype(np.float64)
            gg = g.reshape(-1)[d["idx_" + k]]
        res.append((np.abs(gg - ref).max() / np.abs(ref).max(), k))
    res.sort(reverse=True)
    for r in res[:15]:
        print("%.2e %s" % r)


if __name__ == "__main__":
    main()
