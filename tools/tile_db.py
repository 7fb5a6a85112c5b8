"""Build records/tile_db.txt: the conv tile choices of the engine's autotuner
over the extraction shapes a real stream meets (HPatches / Aachen-like image
sizes at the pipelined loop's batch sizes), run on an MI355X.  The Extractor
loads it at engine creation (posfeat_amd.engine._load_tile_db), so a new image
size reuses the tile of a stored shape within 25 % of its GEMM M instead of
timing every candidate (tiles change speed, never results).

The training step's direct convs (BackboneTrainer, configs[2]) take their
tiles from exact entries of the same file and never time candidates live
(their tiles are not all bit-identical, engine.hip pf_conv_tuned_run); --train
adds those entries: it loads the current database, runs the descriptor-training
step at the bench shapes with POSFEAT_TRAIN_TUNE_LIVE=1 and writes the union.

usage: python tools/tile_db.py [--train] [out]   (GPU box)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TRAIN = "--train" in sys.argv
ARGS = [a for a in sys.argv[1:] if a != "--train"]
if TRAIN:
    os.environ["POSFEAT_TRAIN_TUNE_LIVE"] = "1"   # read once by the library
else:
    os.environ["POSFEAT_TILE_DB"] = "0"   # tune from scratch
# descriptor-training shapes (pairs per GPU, image): the bench line (bs 8) and
# the per-rank half batch of the two-rank SyncBN test
TRAIN_SHAPES = [(8, 480, 640), (4, 480, 640)]

# image sizes: 480x640 .. 880x1200 (HPatches crops, Aachen-like), geometric in
# pixels; batch sizes: the pipelined loop's groups (32) and hold-sized partial
# groups of per-sequence sizes (1 .. 16)
SIZES = [(480, 640), (560, 752), (656, 880), (768, 1024), (880, 1200)]
BATCHES = [1, 2, 4, 6, 8, 12, 16, 24, 32]


def train_main(out):
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.engine import tile_db_export
    from posfeat_amd.training import (BackboneTrainer, DescriptorLossGrad, DESC_EPI_DEFAULTS,
                                      DESC_PRE_DEFAULTS)
    from posfeat_amd.weights import seeded_state_dicts
    bb, _ = seeded_state_dicts(0)
    loss = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
    t0 = time.perf_counter()
    for b, h, w in TRAIN_SHAPES:
        tr = BackboneTrainer(bb, b, h, w, device="cuda:0")
        g = torch.Generator(device="cuda:0").manual_seed(b)
        im1 = torch.rand(b, 3, h, w, device="cuda:0", generator=g) * 4 - 2
        im2 = torch.rand(b, 3, h, w, device="cuda:0", generator=g) * 4 - 2
        F1, F2 = [torch.from_numpy(f).cuda() for f in synthetic_fundamental(b, h, w, 7)]
        t = time.perf_counter()
        tr.step(im1, im2, F1, F2, loss, epoch=1, update=False)
        torch.cuda.synchronize()
        print("train b %d %d x %d  first step %.2f s" % (b, h, w, time.perf_counter() - t),
              flush=True)
        del tr
    n = tile_db_export(out)
    print("%d entries -> %s (%.1f s)" % (n, out, time.perf_counter() - t0))


def main():
    from posfeat_amd.engine import ExtractionEngine, tile_db_export
    from posfeat_amd.weights import seeded_state_dicts
    out = ARGS[0] if ARGS else os.path.join(ROOT, "records", "tile_db.txt")
    if TRAIN:
        return train_main(out)
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
