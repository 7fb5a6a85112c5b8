"""Run the head.conv2-shaped conv (B x 480x640, 3x3, 256->128, NHWC) alone,
for PMC counter passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 480, 640, 256, device="cuda", generator=g)
w = torch.randn(128, 256, 3, 3, device="cuda", generator=g) * 0.03
wp, bp = ops.pack_conv_weight(w, torch.zeros(128, device="cuda"))
y = torch.empty(B, 480, 640, 128, device="cuda")
for _ in range(REPS):
    ops.conv2d_nhwc(x, wp, bp, 128, 3, 3, out=y)
torch.cuda.synchronize()
print("algorithmic bytes/launch: read %.1f MB + write %.1f MB" % (
    x.numel() * 4 / 1e6 + wp.numel() * 4 / 1e6, y.numel() * 4 / 1e6))
