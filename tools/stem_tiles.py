"""Repro tool: the Cin = 4 stem conv (7x7 s2, B=8 480x640) on each register-
staged tile (POSFEAT_CONV_TILE 0 / 1 / 2), one child process each, against
fp64; repeated launches must be bit-equal.  POSFEAT_BF6_STEM=1 selected a
bf16x6 variant of conv_mfma_kernel that was tried and reverted (r6f: its
128x64 tile was not repeatable) -- without it the env
value is ignored and all six runs are the fp32 kernel."""
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd import ops
g = torch.Generator().manual_seed(5)
x = torch.randn(8, 4, 480, 640, generator=g)
wt = torch.randn(64, 4, 7, 7, generator=g) / 14.0
b = torch.randn(64, generator=g) * 0.1
wp, bb = ops.pack_conv_weight(wt.cuda(), b.cuda())
xg = x.permute(0, 2, 3, 1).contiguous().cuda()
ys = [ops.conv2d_nhwc(xg, wp, bb, 64, 7, 7, stride=2).cpu() for _ in range(3)]
assert all(torch.equal(y, ys[0]) for y in ys), "not repeatable"
np.save(%(out)r, ys[0].numpy())
"""
g = torch.Generator().manual_seed(5)
x = torch.randn(8, 4, 480, 640, generator=g)
wt = torch.randn(64, 4, 7, 7, generator=g) / 14.0
b = torch.randn(64, generator=g) * 0.1
ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), stride=2, padding=3)
ref = ref.permute(0, 2, 3, 1).numpy()
for stem in ("0", "1"):
    for tile in ("0", "1", "2"):
        out = "/tmp/stem_%s_%s.npy" % (stem, tile)
        subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "out": out}],
                       env=dict(os.environ, POSFEAT_CONV_TILE=tile, POSFEAT_BF6_STEM=stem),
                       check=True, timeout=120)
        y = np.load(out)
        print("bf6_stem", stem, "tile", tile, "max err %.3e" % np.abs(y - ref).max(), flush=True)
