"""Repro / A-B tool: the B=32 480x640 bench instance against B=1 runs of the
same images (tests/test_gpu_bench_config.py's check), plus run-to-run
repeatability of the B=32 instance.  One child process per variant (env
switches are read once per process).

usage: python tools/b32_repro.py [VARIANT=ENV,ENV ...]
  e.g. python tools/b32_repro.py cur= bf6b=POSFEAT_BF6D=0 r2=POSFEAT_HIP_LIB=ab/lib_r2.so
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import sys, json, numpy as np, torch
sys.path.insert(0, %(root)r)
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.weights import seeded_image, seeded_state_dicts
B, H, W = %(B)d, 480, 640
bb, hd = seeded_state_dicts(0)
imgs = torch.from_numpy(np.stack([seeded_image(i, H, W) for i in range(B)])).cuda()
engB = ExtractionEngine(bb, hd, device="cuda:0")
engB.run(imgs)
runs = []
for r in range(3):
    o = engB.run(imgs)
    runs.append((o["local_point"].clone(), o["local_map"].clone()))
torch.cuda.synchronize()
rep = [max(float((runs[r][0] - runs[0][0]).abs().max()), float((runs[r][1] - runs[0][1]).abs().max()))
       for r in range(1, 3)]
eng1 = ExtractionEngine(bb, hd, device="cuda:0")
errs = []
for i in range(B):
    o1 = eng1.run(imgs[i:i + 1])
    e = float((runs[0][0][i] - o1["local_point"][0]).abs().max())
    s = float(o1["local_point"].abs().max())
    errs.append(e / max(1.0, s))
bad = [i for i, e in enumerate(errs) if e > 1e-4]
print(json.dumps({"repeat_maxdiff": rep, "b1_relerr_max": max(errs), "bad_images": bad[:16],
                  "n_bad": len(bad)}))
"""


def main():
    variants = sys.argv[1:] or ["cur="]
    B = int(os.environ.get("REPRO_B", "32"))
    for v in variants:
        tag, _, envs = v.partition("=")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, val = kv.partition("=")
            env[k] = os.path.join(ROOT, val) if k == "POSFEAT_HIP_LIB" else val
        r = subprocess.run([sys.executable, "-c", CODE % {"root": ROOT, "B": B}], env=env,
                           capture_output=True, text=True, timeout=400)
        out = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-1500:]
        print("[%s] rc=%d %s" % (tag, r.returncode, out), flush=True)
        if r.returncode < 0 or r.returncode >= 124:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
