"""Signed (systematic) error of the dense bf16x6 GEMM tiles against fp64: the
mean of (y - y64) / scale over a large 1x1 conv, for the current build's
dense tiles (POSFEAT_BF6X=0: the 32x32x16 bf6d tiles).  A truncating
accumulation shows up as a mean of the same sign as y; round-to-nearest as
~0.  usage: [POSFEAT_BF6X=0] python tools/bf6_bias.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from posfeat_amd import ops
    from posfeat_amd._lib import lib
    g = torch.Generator().manual_seed(1)
    for cin, cout, h, w in ((512, 256, 64, 80), (192, 192, 48, 52), (1152, 192, 24, 52)):
        x = torch.randn(1, cin, h, w, generator=g).abs() + 0.1  # positive data: a bias adds up
        wt = torch.randn(cout, cin, 1, 1, generator=g) / np.sqrt(cin)
        ref = torch.nn.functional.conv2d(x.double(), wt.double()).permute(0, 2, 3, 1)
        mag = torch.nn.functional.conv2d(x.double(), wt.double().abs()).permute(0, 2, 3, 1)
        xg = x.permute(0, 2, 3, 1).contiguous().cuda()
        wp, bb = ops.pack_conv_weight(wt.cuda(), torch.zeros(cout).cuda())
        pl = ops.split_weight_planes(wp)
        res = {}
        for mode in (1, 0):
            lib().posfeat_set_conv_precision(mode)
            y = (ops.conv2d_nhwc_planes(xg, wp, pl, bb, cout, 1, 1) if mode
                 else ops.conv2d_nhwc(xg, wp, bb, cout, 1, 1)).cpu().double()
            e = (y - ref) / mag
            res[mode] = (float(e.mean()), float((e * torch.sign(ref)).mean()), float(e.abs().max()))
        lib().posfeat_set_conv_precision(1)
        print("K %4d N %3d: bf16x6 mean %+.3e  sign-mean %+.3e  max %.2e | fp32-MFMA mean %+.3e  "
              "sign-mean %+.3e  max %.2e" % ((cin, cout) + res[1] + res[0]))


if __name__ == "__main__":
    main()
