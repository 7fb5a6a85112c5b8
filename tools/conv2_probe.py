"""Run the head.conv2-shaped conv (B x 480x640, 3x3, 256->128, NHWC) alone,
for PMC counter passes (rocprofv3 --pmc ...) and ablation timing.
Prints the mean ms per launch over REPS timed launches (after one warmup)."""
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
ops.conv2d_nhwc(x, wp, bp, 128, 3, 3, out=y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    ops.conv2d_nhwc(x, wp, bp, 128, 3, 3, out=y)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / REPS
flop = 2.0 * B * 480 * 640 * 128 * 256 * 9
print("lib=%s ms/launch=%.3f TFLOP/s=%.1f" % (os.environ.get("POSFEAT_HIP_LIB", "default"), ms,
                                             flop / ms / 1e9))
print("algorithmic bytes/launch: read %.1f MB + write %.1f MB" % (
    x.numel() * 4 / 1e6 + wp.numel() * 4 / 1e6, y.numel() * 4 / 1e6))
