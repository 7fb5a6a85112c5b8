"""extract.py end to end on a synthetic HPatches-layout directory with the
reference's own configs/extract_hpatches.yaml (batch 1, num_pts 8192, 4
loader workers), timed per stage.

Builds <tmp>/data/hpatches-sequences-release/<seq>/{1..6}.ppm from seeded
uint8 noise at HPatches-like sizes (several shapes per run, as the real
dataset has), a checkpoint directory <tmp>/ckpts/keypoint/005 holding the
seeded weights (backbone.pth / localheader.pth; the effective model_config in
<tmp>/ckpts/keypoint/config.yaml, where training writes it), then runs the
Extractor in this fresh process, as a user would: the whole-run rate includes
building the engine and planning/autotuning one instance per image size;
``steady_images_per_s`` counts from the first group of a size met before.
``--passes 2`` adds a second pass in the same process.  ``--timing``: the
reference's serial loop with synchronising per-stage timers.  Prints one JSON
line.

``--sizes 480x640`` (default) builds every image at the metric's size;
``--sizes mixed`` cycles the three HPatches-like sizes below.  After the run
the same process times the kernel path (engine + detector + sampler on
device-resident batches of the pipeline's group size, no I/O, as bench.py's
step) so the line carries ``steady / kernel_path``.

``kernel_path_replay_images_per_s`` replays the run's own group composition
(shapes and counts) on the kernel path, the denominator for mixed sizes.

``--sizes aachen``: an Aachen Day-Night layout (db/*.jpg, query/day/*/*.jpg,
query/night/nexus5x/*.jpg) at the dataset's own image sizes (db 1063x1600 and
1600x1063, queries 1200x1600; cropped to multiples of 16 by the loader as
datasets/aachen.py does), run with the reference's configs/extract_aachen.yaml
(20480 points, nms r 3, thr 0.5, detector_config_query for the queries);
``--seqs`` then counts groups of 14 images (10 db, 3 day, 1 night).

Every run reports ``images_per_s`` (from the Extractor's first image to its
last file) and ``images_per_s_incl_setup`` (construction included: weights,
engine planning, workers).

usage: python tools/extract_e2e.py [--seqs 96] [--sizes 480x640|mixed|hpatches|aachen] [--timing]
                                   [--passes 1] [--no-write]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (h, w) of HPatches-like images (the dataset crops to multiples of 16)
SIZES = [(480, 640), (600, 800), (752, 1000)]


def hpatches_sizes(nseq, seed=7):
    """A distinct size per sequence, as the real HPatches release has (each
    sequence its own camera / crop; datasets/hpatches.py:35-38 crops every
    image to multiples of 16): h in [480, 880], w in [640, 1200], seeded."""
    rs = np.random.RandomState(seed)
    out = []
    while len(out) < nseq:
        s = (16 * rs.randint(30, 56), 16 * rs.randint(40, 76))
        if s not in out:
            out.append(s)
    return out


# Aachen Day-Night image sizes (h, w) before the loader's crop to multiples of 16
AACHEN_DB = [(1063, 1600), (1600, 1063)]
AACHEN_QUERY = (1200, 1600)


def make_aachen(root, ngroups):
    """<root>/data/aachen/images_upright/{db, query/day/milestone, query/night/nexus5x}
    with 10 db, 3 day and 1 night JPEG per group, seeded smooth noise (quality
    95, as the test trees); returns the cropped sizes."""
    from PIL import Image
    base = os.path.join(root, "data", "aachen", "images_upright")
    rs = np.random.RandomState(17)
    sizes = set()
    for g in range(ngroups):
        for sub, n, hw_of in (("db", 10, lambda i: AACHEN_DB[i % 2]),
                              (os.path.join("query", "day", "milestone"), 3, lambda i: AACHEN_QUERY),
                              (os.path.join("query", "night", "nexus5x"), 1, lambda i: AACHEN_QUERY)):
            d = os.path.join(base, sub)
            os.makedirs(d, exist_ok=True)
            for i in range(n):
                h, w = hw_of(g * n + i)
                small = rs.randint(0, 256, (h // 8, w // 8, 3)).astype(np.uint8)
                im = Image.fromarray(small).resize((w, h), Image.BILINEAR)
                im.save(os.path.join(d, "%04d_%d.jpg" % (g, i)), quality=95)
                sizes.add((h - h % 16, w - w % 16))
    return base, sorted(sizes)


def make_dataset(root, nseq, sizes):
    from PIL import Image
    for s in range(nseq):
        h, w = sizes[s % len(sizes)]
        d = os.path.join(root, "data", "hpatches-sequences-release", "v_synth%02d" % s)
        os.makedirs(d, exist_ok=True)
        rs = np.random.RandomState(100 + s)
        base = rs.randint(0, 256, (h // 8, w // 8, 3)).astype(np.uint8)
        for i in range(1, 7):
            im = Image.fromarray(base).resize((w, h), Image.BILINEAR)
            arr = np.asarray(im).astype(np.int16) + rs.randint(-12, 13, (h, w, 3))
            Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8)).save(os.path.join(d, "%d.ppm" % i))


def make_checkpoint(root):
    import torch
    from posfeat_amd.weights import seeded_state_dicts
    ck = os.path.join(root, "ckpts", "keypoint", "005")
    os.makedirs(ck, exist_ok=True)
    bb, hd = seeded_state_dicts(0)
    torch.save(bb, os.path.join(ck, "backbone.pth"))
    torch.save(hd, os.path.join(ck, "localheader.pth"))
    syn = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_synthetic.yaml")))
    yaml.safe_dump({"model": "PoSFeat", "model_config": syn["model_config"]},
                   open(os.path.join(os.path.dirname(ck), "config.yaml"), "w"))


def kernel_path_rate(eng, ex, hw, group, steps=5):
    """bench.py's step (engine + detect + sample, device-resident, no host I/O)
    at this run's group size and first image size, on the run's own engine."""
    import torch
    from posfeat_amd import ops
    from posfeat_amd.weights import seeded_image
    h, w = hw
    cfg = ex.config["detector_config"]
    imgs = torch.from_numpy(np.stack([seeded_image(i, h, w) for i in range(group)])).cuda()
    ws = ops.DetectWorkspace()

    def step():
        out = eng.run(imgs, outputs=())
        _, coord, _, _, n_dev = ops.detect(out["local_point"], cfg["nms_radius"], cfg["num_pts"],
                                           thr=cfg["thr"], thr_mod=cfg["thr_mod"], ws=ws,
                                           sync=False)
        ops.sample_desc_nhwc(out["_local_map_nhwc"], coord, c=128, n_valid=n_dev)
    step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return steps * group / (time.perf_counter() - t)


def kernel_path_replay(eng, ex, groups):
    """The kernel path over this run's own group composition: every group
    (shape, image count) the pipelined loop launched, in order, engine +
    detect_each + sample_each on device-resident seeded images, timed after
    one untimed replay (every shape planned).  Inputs are built before the
    timed region."""
    import torch
    from posfeat_amd import ops
    from posfeat_amd.weights import seeded_image
    cfg = ex.config["detector_config"]
    ins = [torch.from_numpy(np.stack([seeded_image(i, h, w) for i in range(k)])).cuda()
           for (h, w, _), k in groups]

    def replay():
        for imgs in ins:
            out = eng.run(imgs, outputs=())
            _, coord, _, _, n_dev = ops.detect(out["local_point"], cfg["nms_radius"],
                                               cfg["num_pts"], thr=cfg["thr"],
                                               thr_mod=cfg["thr_mod"], sync=False, each=True)
            ops.sample_desc_nhwc(out["_local_map_nhwc"], coord, c=128, n_valid=n_dev, each=True)
    replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    replay()
    torch.cuda.synchronize()
    return sum(k for _, k in groups) / (time.perf_counter() - t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=96)
    ap.add_argument("--sizes", default="480x640",
                    help="HxW, 'mixed' (three sizes cycled) or 'hpatches' (a distinct size per "
                         "sequence)")
    ap.add_argument("--timing", action="store_true", help="per-stage (synchronising) timing")
    ap.add_argument("--passes", type=int, default=1, help="2: a second (warm) pass")
    ap.add_argument("--no-write", action="store_true",
                    help="output_desc: False (no npz files): the run without its file output")
    args = ap.parse_args()
    if args.timing:
        os.environ["POSFEAT_EXTRACT_TIMING"] = "1"
    if args.sizes == "mixed":
        sizes = SIZES
    elif args.sizes == "hpatches":
        sizes = hpatches_sizes(args.seqs)
    elif args.sizes == "aachen":
        sizes = None   # make_aachen's
    else:
        sizes = [tuple(int(v) for v in args.sizes.split("x"))]
    tmp = tempfile.mkdtemp(prefix="posfeat_e2e_")
    t = time.perf_counter()
    aachen = args.sizes == "aachen"
    if aachen:
        data_path, sizes = make_aachen(tmp, args.seqs)
        nimg = 14 * args.seqs
        cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_aachen.yaml")))
        cfg["data_config_extract"]["data_path"] = data_path
    else:
        make_dataset(tmp, args.seqs, sizes)
        nimg = 6 * args.seqs
        cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_hpatches.yaml")))
        cfg["data_config_extract"]["data_path"] = os.path.join(tmp, "data",
                                                               "hpatches-sequences-release")
    print("[e2e] dataset of %d images built in %.1f s" % (nimg, time.perf_counter() - t),
          flush=True)
    make_checkpoint(tmp)
    if args.no_write:
        cfg["output_desc"] = False
    os.chdir(tmp)
    from posfeat_amd.managers.extractor import Extractor
    res = {}
    for p in ("cold", "warm")[:args.passes]:
        cfg["output_root"] = ("aachen/e2e_" if aachen else "hpatches/e2e_") + p
        cp = os.path.join(tmp, "cfg_%s.yaml" % p)
        yaml.safe_dump(cfg, open(cp, "w"))
        t = time.perf_counter()
        ex = Extractor(argparse.Namespace(config=cp, local_rank=-1))
        setup = time.perf_counter() - t
        ex.extract()
        st = dict(ex.stats)
        marks = st.pop("group_marks", None)
        if marks:   # from the first group of a shape met before, to the end
            seen, first = set(), None
            for (t_, k_), shp in zip(marks, ex.group_shapes):
                if shp in seen and first is None:
                    first = (t_, k_)
                seen.add(shp)
            if first is not None:
                st["steady_images_per_s"] = (st["images"] - first[1]) / (st["seconds"] - first[0])
        st["setup_s"] = setup
        st["setup_phases_s"] = {k: round(v, 4) for k, v in getattr(ex, "setup_marks", {}).items()}
        st["images_per_s_incl_setup"] = st["images"] / (st["seconds"] + setup)
        eng = ex.model._engine
        st["kernel_path_images_per_s"] = kernel_path_rate(eng, ex, sizes[0], st.get("group", 32))
        if marks:
            counts = [k for _, k in marks[1:]] + [st["images"]]
            groups = [(shp, c - k) for shp, (_, k), c in zip(ex.group_shapes, marks, counts)]
            st["kernel_path_replay_images_per_s"] = kernel_path_replay(eng, ex, groups)
            st["whole_over_replay"] = st["images_per_s"] / st["kernel_path_replay_images_per_s"]
            st["whole_incl_setup_over_replay"] = (st["images_per_s_incl_setup"]
                                                  / st["kernel_path_replay_images_per_s"])
        if "steady_images_per_s" in st:
            st["steady_over_kernel_path"] = st["steady_images_per_s"] / st["kernel_path_images_per_s"]
            if marks:
                st["steady_over_replay"] = (st["steady_images_per_s"]
                                            / st["kernel_path_replay_images_per_s"])
        st["engine_shapes"] = len(eng.cached_shapes)
        st["engine_stats"] = dict(eng.stats)
        if marks:
            st["groups"] = [[round(t_, 3), k_, list(shp)] for (t_, k_), shp in
                            zip(marks, ex.group_shapes)]
        st["engine_workspace_mb"] = eng.workspace_bytes / 2 ** 20
        res[p] = st
        ex.model._engine = None
        files = []
        for dp, _, fs in os.walk(os.path.join(tmp, "ckpts", cfg["output_root"], "desc")):
            files += [os.path.join(dp, f) for f in fs]
        st["npz_files"] = len(files)
        if files:
            st["kpts_first"] = int(np.load(files[0])["keypoints"].shape[0])
        del ex, eng
        import gc
        import torch
        gc.collect()
        torch.cuda.empty_cache()
    import torch
    if aachen:
        data = "synthetic Aachen Day-Night layout, %d groups x (10 db + 3 day + 1 night) jpg, " \
               "cropped sizes %s" % (args.seqs, sizes)
    else:
        data = "synthetic HPatches layout, %d seqs x 6 ppm, sizes %s" % (
            args.seqs, sorted({sizes[s % len(sizes)] for s in range(args.seqs)}))
    print(json.dumps({"workload": "extract.py e2e (configs/extract_%s.yaml: loader batch 1 "
                                  "in the reference; the pipelined loop groups by shape)"
                                  % ("aachen" if aachen else "hpatches"),
                      "data": data,
                      "device": torch.cuda.get_device_name(0), **res}))


if __name__ == "__main__":
    main()
