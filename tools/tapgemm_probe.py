"""Dense pre-split-weight GEMM timing on the extraction's dominant shapes:
head.conv2's tap GEMM (B x 120 x 160 x 192 -> 1152) and a 512 -> 256 1x1
of the decoder F(6x6) GEMMs' size, one tile (conv2d_nhwc_planes), HIP
events over REPS launches.  A/B switches (POSFEAT_BF6X_MEMF ...) need the A/B
library (POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so).  PROBE_SHAPES=enc:
the encoder's short-K 1x1 convs instead.
usage: python tools/tapgemm_probe.py [tile] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd import ops  # noqa: E402

TILE = int(sys.argv[1]) if len(sys.argv) > 1 else 29
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
SHAPES = [("tap", 32, 120, 160, 192, 1152), ("f6", 64, 120, 144, 512, 256)]
if os.environ.get("PROBE_SHAPES") == "enc":   # the encoder's short-K 1x1 convs at B = 32
    SHAPES = [("l3conv3", 32, 30, 40, 256, 1024), ("l2conv3", 32, 60, 80, 128, 512),
              ("l3conv1", 32, 30, 40, 1024, 256), ("l2conv1", 32, 60, 80, 512, 128),
              ("l1conv1", 32, 120, 160, 256, 64)]
g = torch.Generator(device="cuda").manual_seed(0)
for name, n, h, w, cin, cout in SHAPES:
    x = torch.randn(n, h, w, cin, device="cuda", generator=g)
    wt = torch.randn(cout, cin, 1, 1, device="cuda", generator=g) / cin ** 0.5
    wp, bp = ops.pack_conv_weight(wt, torch.zeros(cout, device="cuda"))
    planes = ops.split_weight_planes(wp)
    y = torch.empty(n, h, w, cout, device="cuda")
    ops.conv2d_nhwc_planes(x, wp, planes, bp, cout, 1, 1, out=y, tile=TILE)
    torch.cuda.synchronize()
    ref = y.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        ops.conv2d_nhwc_planes(x, wp, planes, bp, cout, 1, 1, out=y, tile=TILE)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / REPS
    tf = 2.0 * n * h * w * cin * cout / ms / 1e9
    print("%s tile %d: %.3f ms  %.1f TF/s  frac %.3f  repeat %s" % (
        name, TILE, ms, tf, tf / 416.7,
        bool(torch.equal(ref, y))), flush=True)
