"""Every legal conv tile on a set of conv shapes: bit-equal repeated launches
and the error against an fp64 reference (the repeatability sweep behind
tests/test_gpu_tiles.py).  One child process per tile (POSFEAT_CONV_TILE is
read once per process).

usage: python tools/tile_sweep.py [--tiles 0,1,2,...] [--lib path]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (n, h, w, cin, cout, k, stride): the stem, a 1x1, a strided 1x1, a 3x3 s1,
# a 3x3 s2, a short-K 1x1 at the bench batch's layer1 scale
SHAPES = [(8, 240, 320, 4, 64, 7, 2), (8, 120, 160, 256, 64, 1, 1), (8, 120, 160, 256, 512, 1, 2),
          (8, 60, 80, 128, 128, 3, 1), (8, 120, 160, 128, 128, 3, 2), (32, 120, 160, 64, 256, 1, 1)]
TILES = [0, 1, 2, 3, 10, 11, 12, 20, 21, 22, 23]

CODE = r"""
import sys, json, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd import ops
res = []
for (n, h, w, cin, cout, k, s) in %(shapes)r:
    g = torch.Generator().manual_seed(n * h + cin + k)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    wp, bb = ops.pack_conv_weight(wt.cuda(), b.cuda())
    xg = x.permute(0, 2, 3, 1).contiguous().cuda()
    if cin %% 4:
        xg = torch.nn.functional.pad(xg, (0, 4 - cin %% 4))
    try:
        ys = [ops.conv2d_nhwc(xg, wp, bb, cout, k, k, stride=s, cin=cin) for _ in range(3)]
    except RuntimeError as e:
        res.append({"shape": [n, h, w, cin, cout, k, s], "skip": str(e)[:80]})
        continue
    torch.cuda.synchronize()
    rep = max(float((y - ys[0]).abs().max()) for y in ys[1:])
    sub = slice(0, 2)
    ref = torch.nn.functional.conv2d(x[sub].double(), wt.double(), b.double(), stride=s,
                                     padding=(k - 1) // 2).permute(0, 2, 3, 1)
    scale = torch.nn.functional.conv2d(x[sub].double().abs(), wt.double().abs(), None, stride=s,
                                       padding=(k - 1) // 2).permute(0, 2, 3, 1).max()
    err = float((ys[0][sub].cpu().double() - ref).abs().max() / scale)
    res.append({"shape": [n, h, w, cin, cout, k, s], "repeat_maxdiff": rep, "err_rel": err})
print(json.dumps(res))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default=",".join(map(str, TILES)))
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    bad = 0
    for t in [int(v) for v in args.tiles.split(",")]:
        env = dict(os.environ, POSFEAT_CONV_TILE=str(t))
        if args.lib:
            env["POSFEAT_HIP_LIB"] = os.path.join(ROOT, args.lib)
        r = subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "shapes": SHAPES}],
                           env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print("tile %d rc=%d %s" % (t, r.returncode, r.stderr[-800:]), flush=True)
            if r.returncode < 0 or r.returncode >= 124:
                return 2
            continue
        for rec in json.loads(r.stdout.strip().splitlines()[-1]):
            flag = ""
            if rec.get("repeat_maxdiff", 0) != 0 or rec.get("err_rel", 0) > 1e-5:
                flag = "  <-- BAD"
                bad += 1
            print("tile %2d %s%s" % (t, json.dumps(rec), flag), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
