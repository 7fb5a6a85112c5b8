"""head.conv2 by bilinear phases (posfeat_conv2_up4) alone at B x 480x640, for
rocprofv3 kernel traces: prints ms per call (weights build + border + main +
statistics) over REPS timed calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H, W = 480, 640
g = torch.Generator(device="cuda").manual_seed(0)
L = torch.randn(B, H // 4, W // 4, 192, device="cuda", generator=g)
G = torch.randn(B, H, W, 64, device="cuda", generator=g)
w = torch.randn(128, 256, 3, 3, device="cuda", generator=g) * 0.03
wp, bp = ops.pack_conv_weight(w, torch.zeros(128, device="cuda"))
y = torch.empty(B, H, W, 128, device="cuda")
ops.conv2_up4_instnorm_stats(L, G, wp, bp, out=y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    ops.conv2_up4_instnorm_stats(L, G, wp, bp, out=y)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / REPS
print("up4 ms/call=%.3f  reference-conv TFLOP/s=%.1f" % (ms, 2.0 * B * H * W * 128 * 2304 / ms / 1e9))
