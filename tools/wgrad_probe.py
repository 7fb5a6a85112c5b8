"""head.conv2 weight gradient (posfeat_conv_wgrad, 256 -> 128, 3x3) alone at
B x 480x640 for timing / rocprofv3 counter passes: prints ms per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd._lib import check, lib, ptr, stream_ptr  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
CIN = int(sys.argv[3]) if len(sys.argv) > 3 else 256
COUT = int(sys.argv[4]) if len(sys.argv) > 4 else 128
H, W = (int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else (480, 640)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, H, W, CIN, device="cuda", generator=g)
dy = torch.randn(B, H, W, COUT, device="cuda", generator=g)
kpad = lib().posfeat_conv_packed_k(CIN, 3, 3)
dw = torch.empty(COUT * kpad, device="cuda")
db = torch.empty(COUT, device="cuda")
need = lib().posfeat_conv_wgrad_workspace(B, H, W, CIN, COUT, 3, 3)
ws = torch.empty(need, dtype=torch.uint8, device="cuda")


def run():
    check(lib().posfeat_conv_wgrad(ptr(dy), COUT, ptr(x), CIN, B, H, W, CIN, COUT, 3, 3, ptr(dw),
                                   ptr(db), ptr(ws), need, stream_ptr()))


run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / REPS
fl = 2.0 * B * H * W * COUT * CIN * 9
print("wgrad B=%d %dx%d %d->%d: %.3f ms/call  %.1f TFLOP/s" % (B, H, W, CIN, COUT, ms, fl / ms / 1e9))
