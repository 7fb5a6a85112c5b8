"""Forward timing of the training-side correlation path (BASELINE configs[2]
and [4] shapes): Preprocess_Line2Window + EpipolarLoss_full on B=8 pairs of
480x640 (desc training, train_desc.yaml) and DiskLoss on B pairs
(train_kp.yaml).  Synthetic local maps / score maps / fundamental matrices.

Usage: python tools/bench_correlation.py [batch] [steps]
Prints one JSON line with ms per call for each loss and the oracle (torch
CPU) time of one pair for reference.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from posfeat_amd.correlation import synthetic_fundamental  # noqa: E402
from posfeat_amd.losses import DiskLoss, EpipolarLoss_full, Preprocess_Line2Window  # noqa: E402
from test_gpu_correlation import DESC_CFG, DISK_CFG, EPI_CFG  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    H, W = 480, 640
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    xf1 = torch.randn(B, 128, H // 4, W // 4, device=dev, generator=g)
    xf2 = torch.randn(B, 128, H // 4, W // 4, device=dev, generator=g)
    kp1 = torch.rand(B, 1, H, W, device=dev, generator=g) * 3
    kp2 = torch.rand(B, 1, H, W, device=dev, generator=g) * 3
    F1, F2 = synthetic_fundamental(B, H, W, 0)
    inputs = {"im1": torch.zeros(B, 3, H, W), "im2": torch.zeros(B, 3, H, W),
              "F1": torch.from_numpy(F1).to(dev), "F2": torch.from_numpy(F2).to(dev)}
    outputs = {"preds1": {"local_map": xf1, "local_point": kp1},
               "preds2": {"local_map": xf2, "local_point": kp2}, "epoch": 0}
    pre, epi, disk = Preprocess_Line2Window(DESC_CFG), EpipolarLoss_full(EPI_CFG), DiskLoss(DISK_CFG)
    res = {}
    for name, fn in (("line2window+epipolar", lambda: epi(inputs, outputs, pre(inputs, outputs))),
                     ("diskloss", lambda: disk(inputs, outputs, None))):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 3)
    # algorithmic work: cos-sim 2*B*1200^2*128; DiskLoss 2*B*4800^2*128
    res["line2window_cos_gflop"] = 2 * B * 1200 ** 2 * 128 / 1e9
    res["diskloss_gemm_gflop"] = 2 * B * 4800 ** 2 * 128 / 1e9
    res["batch_pairs"] = B
    print(json.dumps(res))


if __name__ == "__main__":
    main()
