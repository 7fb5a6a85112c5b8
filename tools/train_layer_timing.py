"""Per-label timing of one descriptor-training step (bench.py --workload
train_desc's configuration: bs 8 pairs, 480x640): every conv-class label
("fwd:conv:<layer>", "bwd:wgrad:<layer>", "bwd:dgrad:<layer>") with its
milliseconds, launches and TFLOP/s (executed flops), largest first, then the
class totals.  Usage: python tools/train_layer_timing.py [pairs]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from posfeat_amd.correlation import synthetic_fundamental  # noqa: E402
from posfeat_amd.training import (BackboneTrainer, DescriptorLossGrad, DESC_EPI_DEFAULTS,  # noqa: E402
                                  DESC_PRE_DEFAULTS)
from posfeat_amd.weights import seeded_state_dicts  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W = 480, 640
dev = torch.device("cuda", 0)
bb, _ = seeded_state_dicts(0)
tr = BackboneTrainer(bb, b, H, W, device=dev, lr=1e-4)
loss = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
im1 = bench.make_images(0, b, dev)
im2 = bench.make_images(b, b, dev)
F1, F2 = [torch.from_numpy(f).to(dev) for f in synthetic_fundamental(b, H, W, 200)]
for _ in range(3):
    tr.step(im1, im2, F1, F2, loss, epoch=1)
tr.set_timing(True)
tr.step(im1, im2, F1, F2, loss, epoch=1)
by = {}
for lab, ms, fl in tr.timing_events():
    e = by.setdefault(lab, [0.0, 0.0, 0])
    e[0] += ms
    e[1] += fl
    e[2] += 1
tr.set_timing(False)
tot = sum(v[0] for v in by.values())
print("step kernels %.3f ms (timed labels)" % tot)
print("%-40s %8s %6s %8s" % ("label", "ms", "calls", "TFLOP/s"))
for k, v in sorted(by.items(), key=lambda kv: -kv[1][0]):
    print("%-40s %8.3f %6d %8.1f" % (k, v[0], v[2], v[1] / max(v[0], 1e-9) / 1e9))
