"""Per-launch timing of one engine forward (HIP events around every launch
on the engine's stream).  Usage: python tools/layer_timing.py [batch] [h] [w]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posfeat_amd import _lib  # noqa: E402
from posfeat_amd.engine import ExtractionEngine  # noqa: E402
from posfeat_amd.weights import seeded_image, seeded_state_dicts  # noqa: E402


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    w = int(sys.argv[3]) if len(sys.argv) > 3 else 640
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd)
    img = torch.from_numpy(np.stack([seeded_image(i, h, w) for i in range(b)])).cuda()
    for _ in range(2):
        eng.run(img)
    eng.set_timing(b, h, w, True)
    eng.run(img)
    torch.cuda.synchronize()
    handle = eng._instance(b, h, w)[0]
    # walk the labels by querying each distinct prefix
    m = eng._inst[(b, h, w)]
    labels = []
    L = _lib.lib()
    # read back the individual events through the prefix API: rebuild names
    # from the engine layer table + fixed non-conv labels
    names = ["conv:" + s[0] for s in _lib.model_specs() if s[0] != "head.prelu"]
    names += ["layout:", "maxpool", "upsample2x", "instnorm", "instnorm_apply",
              "norm_prelu_up4", "head_tail", "global_feat"]
    tot_ms, _, _ = eng.timing(b, h, w, "")
    rows = []
    for n in names:
        ms, fl, k = eng.timing(b, h, w, n)
        if k == 0:
            continue
        if n.startswith("conv:") and any(o != n and o.startswith(n) for o in names):
            # exact label: 'conv:layer1.0.conv1' is a prefix of nothing else
            pass
        rows.append((ms, n, k, fl / (ms * 1e-3) / 1e12 if ms > 0 and fl > 0 else 0.0))
    rows.sort(reverse=True)
    print("total %.3f ms for batch %d (%dx%d) = %.3f ms/image" % (tot_ms, b, h, w, tot_ms / b))
    print("%-28s %6s %9s %8s %7s" % ("label", "calls", "ms", "TFLOP/s", "share"))
    for ms, n, k, tf in rows:
        print("%-28s %6d %9.3f %8.1f %6.1f%%" % (n, k, ms, tf, 100 * ms / tot_ms))


if __name__ == "__main__":
    main()
