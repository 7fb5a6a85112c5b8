"""Build records/tile_db.txt: the conv tile choices of the engine's autotuner
over the extraction shapes a real stream meets (HPatches / Aachen-like image
sizes at the pipelined loop's batch sizes), run on an MI355X.  The Extractor
loads it at engine creation (posfeat_amd.engine._load_tile_db), so a new image
size reuses the tile of a stored shape within 25 % of its GEMM M instead of
timing every candidate (tiles change speed, never results).

usage: python tools/tile_db.py [out]   (GPU box)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

os.environ["POSFEAT_TILE_DB"] = "0"   # tune from scratch

# image sizes: 480x640 .. 880x1200 (HPatches crops, Aachen-like), geometric in
# pixels; batch sizes: the pipelined loop's groups (32) and hold-sized partial
# groups of per-sequence sizes (1 .. 16)
SIZES = [(480, 640), (560, 752), (656, 880), (768, 1024), (880, 1200)]
BATCHES = [1, 2, 4, 6, 8, 12, 16, 24, 32]


def main():
    from posfeat_amd.engine import ExtractionEngine, tile_db_export
    from posfeat_amd.weights import seeded_state_dicts
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "records", "tile_db.txt")
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device="cuda:0")
    t0 = time.perf_counter()
    for b in BATCHES:
        for h, w in SIZES:
            img = torch.rand(b, 3, h, w, device="cuda:0") * 4 - 2   # random: DVFS ranks tiles as in use
            t = time.perf_counter()
            eng.run(img, outputs=())
            torch.cuda.synchronize()
            print("b %2d %4d x %4d  first forward %.2f s" % (b, h, w, time.perf_counter() - t),
                  flush=True)
    n = tile_db_export(out)
    print("%d entries -> %s (%.1f s)" % (n, out, time.perf_counter() - t0))


if __name__ == "__main__":
    main()
