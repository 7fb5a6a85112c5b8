"""Per-launch timing of one engine forward (HIP events around every launch
on the engine's stream; side-stream launches carry the "side:" prefix and
overlap the main stream).  Usage: python tools/layer_timing.py [batch] [h] [w]"""
import os
import sys
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd.engine import ExtractionEngine  # noqa: E402
from posfeat_amd.weights import seeded_image, seeded_state_dicts  # noqa: E402


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    w = int(sys.argv[3]) if len(sys.argv) > 3 else 640
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd)
    img = torch.from_numpy(np.stack([seeded_image(i, h, w) for i in range(b)])).cuda()
    for _ in range(3):
        eng.run(img)
    eng.set_timing(b, h, w, True)
    eng.run(img)
    torch.cuda.synchronize()
    agg = OrderedDict()
    for lab, ms, fl in eng.timing_events(b, h, w):
        a = agg.setdefault(lab, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += ms
        a[2] += fl
    main_ms = sum(v[1] for k, v in agg.items() if not k.startswith("side:"))
    side_ms = sum(v[1] for k, v in agg.items() if k.startswith("side:"))
    print("main stream %.3f ms, side stream %.3f ms for batch %d (%dx%d) = %.3f ms/image (main)"
          % (main_ms, side_ms, b, h, w, main_ms / b))
    print("%-32s %6s %9s %8s %7s" % ("label", "calls", "ms", "TFLOP/s", "share"))
    for lab, (k, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 and fl > 0 else 0.0
        print("%-32s %6d %9.3f %8.1f %6.1f%%" % (lab, k, ms, tf, 100 * ms / main_ms))


if __name__ == "__main__":
    main()
