"""Benchmark: images/s of the PoSFeat extraction hot path on MI355X.

Metric (BASELINE.json): "images/sec extract (640x480, 2048 kp) at 1/2/4/8 GPU".
One step = one batch of B synthetic 480x640 images (device-resident before the
timed region) through the full extraction path of Extractor.process:
  PoSFeat.extract (ResUNet + KeypointDet, HIP engine)
  -> generate_kpts_single (nms_radius 1, thr 0.9 abs, num_pts 2048; HIP detector)
  -> sample_feat_by_coord (+L2; HIP sampler)
No host synchronisation inside a step (the keypoint count stays on the device).

Multi-GPU: one process per GPU.  ``--gpus N`` (N > 1) without a torchrun
environment makes this process a launcher: before any GPU call it starts N
worker processes of this same script with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set (torchrun's contract, so a torchrun
launch works the same way) and exits with the workers' status.  Each worker
binds cuda:LOCAL_RANK, joins the RCCL process group, receives rank 0's packed
weights by ONE broadcast over xGMI and extracts its own image shard with no
data-path collective ("weak" scaling).  Timing: barrier + synchronize on both
sides of exactly K steps, max over ranks; rank 0 prints the JSON line with
``ranks_seen`` = dist.get_world_size().
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

H, W = 480, 640
NUM_PTS, NMS_R, THR = 2048, 1, 0.9
# images per GPU per extraction step (one engine instance, autotuned at this
# shape; tests/test_gpu_bench_config.py checks this instance image by image)
EXTRACT_BATCH = 32

# Conv work per 480x640 image: 2 x 208.99 GMAC
CONV_FLOP_PER_IMAGE = 417.98e9
HEAD_CONV2_FLOP_PER_IMAGE = 2.0 * 480 * 640 * 128 * 256 * 9   # reference layer
# dominant kernel (roofline): the single MFMA launch with the largest time in
# the step, over EVERY main-stream conv label the engine times (the batched
# Winograd GEMMs of the decoder and the encoder, head.conv2's low-res tap GEMM,
# the 1x1 / strided / halo convs, the stem).  The engine's timing events carry
# the FLOPs each launch executes.
GEMM_LABEL_KERNELS = {
    ".wino": "conv_bf6x_kernel<128> x64 batched (Winograd F(6x6) transform-domain GEMMs of "
             "%s; bf16x6 on pre-split U planes, v_mfma_f32_16x16x32_bf16, memory instructions "
             "interleaved among the MFMAs)",
    "up4tap": "gemm_ws_kernel<1,12,6,8> (head.conv2's 192 x4-upsampled channels: nine 1x1 "
              "convs on the 120x160 grid as one [B*19200 x 192] x [192 x 1152] GEMM; persistent, "
              "each block's 128 x 192 weight planes resident in LDS)",
    "": "the autotuned conv tile of %s (conv.hip MFMA implicit GEMM)",
}
# conv labels whose kernels keep fp32-input MFMA in every precision mode (none
# since the 7x7 stem runs bf16x6 on the bf6x tile's tap gather, round 3)
FP32_MFMA_LABELS = ()
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md, dense FP32 matrix (spec)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md, dense BF16 matrix (no sparsity)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md, HBM3E (~8 TB/s)


def conv_arithmetic():
    """The row-tile convs' product arithmetic (posfeat_set_conv_precision):
    bf16x6 runs each fp32 product as 6 bf16 MFMA products (fp32-accurate,
    tests/test_gpu_precision.py), so its own ceiling is the dense bf16 peak / 6
    in fp32-equivalent FLOP/s."""
    from posfeat_amd._lib import lib
    mode = lib().posfeat_set_conv_precision(-1)
    if mode >= 1:
        return {"arithmetic": "bf16x6: fp32 operands split exactly into 3 bf16 terms, 6 products "
                              "per fp32 product on the bf16 MFMAs (16x16x32 dense GEMMs, 32x32x16 other convs), fp32 accumulate "
                              "(per-product error < one fp32 rounding)",
                "method_peak": round(PEAK_BF16_MFMA_TFLOPS / 6, 1)}
    return {"arithmetic": "fp32-input MFMA v_mfma_f32_32x32x2_f32", "method_peak":
            PEAK_FP32_MFMA_TFLOPS}


def launch_ceiling(mask):
    """(peak TFLOP/s, arithmetic) for a timing label's PF_ARITH mask
    (posfeat_*_timing_event_arith: 1 fp32 MFMA, 2 bf16x6, 3 both).  A label
    mixing both is priced against the higher (bf16x6) ceiling, the stricter
    fraction."""
    if mask & 2:
        return round(PEAK_BF16_MFMA_TFLOPS / 6, 1), ("bf16x6" if mask == 2 else
                                                     "bf16x6 + fp32 MFMA (priced at bf16x6)")
    return PEAK_FP32_MFMA_TFLOPS, "fp32 MFMA (v_mfma_f32_32x32x2_f32)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None,
                   help="images (extract) or pairs (training workloads) per GPU per step; "
                        "default: %d images for extract (r5c sweep on one box: B=8 847, 16 890, "
                        "32 939, 48 947, 64 951 img/s -- the layer3/decoder grids fill at 32; "
                        "r6g same box: 32 946.9, 64 963.0, but at 64 the side stream's "
                        "K=80 conv overlaps a decoder GEMM, see DESIGN 4.1m), "
                        "8 pairs for the training workloads (configs[2]: bs=8)" % EXTRACT_BATCH)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="extract: skip the corr / train_kp / train_desc lines timed after the "
                        "headline loop (N=1 only)")
    p.add_argument("--secondary-steps", type=int, default=10)
    p.add_argument("--graph", action="store_true",
                   help="extract: replay the step as one captured hipGraph (r3n: 798.4 vs "
                        "798.2 img/s eager -- the step is not launch-bound)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--timing-steps", type=int, default=3)
    p.add_argument("--master-port", type=int, default=0,
                   help="rendezvous port for the --gpus N launcher (0: pick a free one)")
    p.add_argument("--workload", choices=("extract", "train_kp", "train_desc", "corr", "stub"),
                   default="extract",
                   help="extract: configs[1] (the metric); train_kp: configs[4], the keypoint-"
                        "head training step (DiskLoss); train_desc: configs[2], the descriptor "
                        "training step (backbone, Line2Window + EpipolarLoss, Adam); training "
                        "workloads use --batch pairs per GPU; corr: the correlation losses of "
                        "configs[2] and [4] (Line2Window + EpipolarLoss and DiskLoss, value + "
                        "map gradients) on synthetic maps; stub: a CPU-only step over "
                        "gloo that tests the launcher and the timing protocol")
    args = p.parse_args()
    if args.batch is None:
        args.batch = EXTRACT_BATCH if args.workload == "extract" else 8
    return args


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(args, argv=None):
    """--gpus N > 1 without WORLD_SIZE in the environment: start N fresh
    worker processes of this script (one per GPU, torchrun's environment
    contract) and return their combined exit status.  Runs before anything
    touches the GPU (no torch.cuda call in this process), and starts the
    workers as children instead of exec-ing.  A failed worker stops the
    others, so no rank waits forever in a collective."""
    argv = sys.argv[1:] if argv is None else argv
    n = args.gpus
    port = args.master_port or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    status = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            rc = p.poll()
            if rc is None:
                continue
            alive.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in alive:
                    q.terminate()
        time.sleep(0.05)
    return status


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if args.workload == "stub":
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def ranks_seen():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def timed_loop(world, steps, fn, sync):
    """barrier + sync, exactly ``steps`` calls of fn, sync + barrier; max over ranks."""
    import torch.distributed as dist
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def stub_main(args, world, rank):
    """CPU-only stand-in step (a small matmul per rank) for the launcher test:
    same launch, barrier/timing protocol and JSON line as the real workloads."""
    g = torch.Generator().manual_seed(rank)
    a = torch.rand(128, 128, generator=g)

    def one():
        torch.mm(a, a)
    for _ in range(args.warmup):
        one()
    el = timed_loop(world, args.steps, one, lambda: None)
    if rank == 0:
        print(json.dumps({"metric": "stub steps/s", "value": round(world * args.steps / el, 3),
                          "unit": "steps/s", "n_gpus": world, "ranks_seen": ranks_seen(),
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak"}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def build_engine(world, rank, dev, train=False):
    """Rank 0 packs the seeded weights; one RCCL broadcast ships the blob."""
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd import _lib, weights
    nfl = _lib.lib().posfeat_model_weight_floats()
    if rank == 0:
        bb, hd = weights.seeded_state_dicts(0)
        blob = torch.from_numpy(weights.pack_for_device(bb, hd, _lib.model_specs()))
        buf = torch.zeros(nfl, dtype=torch.float32, device=dev)
        buf[:blob.numel()].copy_(blob.to(dev))
    else:
        buf = torch.empty(nfl, dtype=torch.float32, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(buf, src=0)
    return ExtractionEngine(device=dev, blob=buf, train=train)


def make_images(rank, batch, dev):
    from posfeat_amd.weights import seeded_image
    ims = [seeded_image(rank * batch + i, H, W) for i in range(batch)]
    return torch.from_numpy(np.stack(ims)).to(dev)


# PoSFeat.extract's engine outputs (networks/PoSFeat_model.py: local_map,
# global_map, global_feat, local_point; local_map_small feeds the head only)
EXTRACT_OUTPUTS = ("local_map", "global_map", "global_feat")


def step(engine, ops, ws, imgs):
    """PoSFeat.extract + Extractor.process for one batch: the engine with the
    NCHW outputs and global_feat PoSFeat.extract returns (plus its local_thr /
    global_point constants), the detector and the descriptor sampler."""
    out = engine.run(imgs, outputs=EXTRACT_OUTPUTS)
    lp = out["local_point"]
    b, _, h, w = out["global_map"].shape
    out["local_thr"] = torch.zeros_like(lp)
    out["global_point"] = torch.ones(b, 1, h, w, device=lp.device)
    idx, coord, score, counts, n_dev = ops.detect(lp, NMS_R, NUM_PTS, thr=THR,
                                                  thr_mod="abs", ws=ws, sync=False)
    desc = ops.sample_desc_nhwc(out["_local_map_nhwc"], coord, c=128, n_valid=n_dev)
    return desc, coord, score


def host_cpu_info():
    """nproc, the CPUs this process may run on, and the CPU model."""
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return os.cpu_count() or 1, avail, model


def cpu_baseline(seconds):
    """Oracle (torch-CPU restatement of the reference path) on host cores."""
    from oracle import model_ref, detect_ref
    from posfeat_amd.weights import seeded_state_dicts, seeded_image
    nproc, avail, model = host_cpu_info()
    # every CPU this process may use; OMP_NUM_THREADS (set to the box's CPU
    # share by the GPU pool) caps it, since threads beyond the share only
    # time-slice against each other
    threads = avail
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, max(1, int(os.environ["OMP_NUM_THREADS"])))
    torch.set_num_threads(threads)
    bb, hd = seeded_state_dicts(0)

    def one(i):
        img = torch.from_numpy(seeded_image(i, H, W))[None]
        o = model_ref.posfeat_extract(bb, hd, img)
        detect_ref.process_image(o["local_point"].numpy(), o["local_map"].numpy(),
                                 dict(nms_radius=NMS_R, num_pts=NUM_PTS, thr=THR, thr_mod="abs"),
                                 H, W)
    one(0)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        one(n + 1)
        n += 1
        el = time.perf_counter() - t0
        if el > seconds or n >= 30:
            break
    return {"value": n / el, "unit": "images/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cpus_available": avail, "cpu_model": model,
            "sample": "%d seeded 480x640 images, extract+detect(2048)+sample, batch 1, "
                      "torch-CPU oracle (oracle/model_ref.py + oracle/detect_ref.py)" % n}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args))
    world, rank, local = setup_dist(args)
    if args.workload == "stub":
        return stub_main(args, world, rank)
    dev = torch.device("cuda", local if world > 1 else torch.cuda.current_device())
    torch.cuda.set_device(dev)
    if args.workload == "train_kp":
        return train_main(args, world, rank, dev)
    if args.workload == "train_desc":
        return train_desc_main(args, world, rank, dev)
    if args.workload == "corr":
        return corr_main(args, world, rank, dev)
    from posfeat_amd import ops
    import torch.distributed as dist
    engine = build_engine(world, rank, dev)
    ws = ops.DetectWorkspace()
    imgs = make_images(rank, args.batch, dev)
    for _ in range(args.warmup):
        step(engine, ops, ws, imgs)
    # --graph: the step as ONE hipGraph (torch.cuda.CUDAGraph over the engine's
    # stream; the side stream joins the capture through the engine's fork/join
    # events): every replay launches every kernel of the step again on the
    # same resident inputs -- no work is cached -- without the ~150 host
    # launches.  Measured no faster (the GPU, not the host, paces the step), so
    # the default is eager; the eager rate is always reported.
    eager_steps = max(1, min(args.steps, 20))
    el_eager = timed_loop(world, eager_steps, lambda: step(engine, ops, ws, imgs),
                          torch.cuda.synchronize)
    run = lambda: step(engine, ops, ws, imgs)
    launch = "eager"
    if args.graph:
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step(engine, ops, ws, imgs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            step(engine, ops, ws, imgs)
        graph.replay()
        torch.cuda.synchronize()
        run = graph.replay
        launch = "hipGraph replay of the captured step"
    el = timed_loop(world, args.steps, run, torch.cuda.synchronize)
    images = world * args.steps * args.batch
    value = images / el

    # ---- roofline of the dominant kernel, HIP events on the engine's stream
    # around each launch, averaged over a few extra steps
    engine.set_timing(args.batch, H, W, True)
    per_label, other_ms = {}, {}
    c2_ms, conv_ms, conv_fl, all_ms, side_ms = [], [], [], [], []
    for _ in range(args.timing_steps):
        step(engine, ops, ws, imgs)
        ev = engine.timing_events(args.batch, H, W)
        for lab, ms, fl in ev:
            if lab.startswith("conv:") and fl > 0:
                per_label.setdefault(lab, []).append((ms, fl))
            elif not lab.startswith(("conv:", "side:")):
                other_ms.setdefault(lab, []).append(ms)
        main = [e for e in ev if not e[0].startswith("side:")]
        c2_ms.append(sum(ms for lab, ms, _ in main if lab.startswith(("conv:head.conv2",
                                                                        "head.conv2"))))
        conv_ms.append(sum(ms for lab, ms, _ in main if lab.startswith("conv:")))
        conv_fl.append(sum(fl for lab, _, fl in main if lab.startswith("conv:")))
        all_ms.append(sum(ms for _, ms, _ in main))
        side_ms.append(sum(ms for lab, ms, _ in ev if lab.startswith("side:")))
    engine.set_timing(args.batch, H, W, False)
    dom = max(per_label, key=lambda k: np.mean([m for m, _ in per_label[k]]))
    kms = float(np.mean([m for m, _ in per_label[dom]]))
    k_flops = float(np.mean([f for _, f in per_label[dom]]))
    achieved = k_flops / (kms * 1e-3) / 1e12
    kkey = next(k for k in GEMM_LABEL_KERNELS if dom.endswith(k))
    kdesc = GEMM_LABEL_KERNELS[kkey]
    if "%s" in kdesc:
        kdesc = kdesc % (dom[len("conv:"):-len(kkey)] if kkey else dom[len("conv:"):])
    arith = conv_arithmetic()
    if dom in FP32_MFMA_LABELS:   # this launch runs fp32-input MFMA whatever the mode
        arith = {"arithmetic": "fp32-input MFMA v_mfma_f32_32x32x2_f32",
                 "method_peak": PEAK_FP32_MFMA_TFLOPS}
    c2 = float(np.mean(c2_ms))
    conv_total = float(np.mean(conv_ms))
    conv_ach = float(np.mean(conv_fl)) / (conv_total * 1e-3) / 1e12
    # HBM bytes of that launch from the committed rocprofv3 --pmc passes
    # (tools/traffic_json.py), when they were measured for the same label;
    # records/ travels to the GPU box (profiles/ does not)
    traffic = None
    tfile = os.path.join(ROOT, "records", "dominant_traffic.json")
    if os.path.exists(tfile):
        try:
            recs = json.load(open(tfile))
            for t in recs.get("records", [recs]):  # one record or {"records": [...]}
                if dom in t.get("labels", []) and t.get("batch") == args.batch:
                    traffic = t.get("bytes_per_launch")
                    break
        except Exception:
            traffic = None

    # the longest non-GEMM launch (head.conv2's tap combine with the
    # folded image conv, up4tap_gcombine_kernel) against the HBM roofline:
    # algorithmic bytes = the tap maps P read once (B h w 1152 fp32) + y written
    # once (B H W 128 fp32) + the NHWC4 image read once
    hb = max(other_ms, key=lambda k: np.mean(other_ms[k]))
    hb_ms = float(np.mean(other_ms[hb]))
    hb_rec = {"label": hb, "avg_launch_ms": round(hb_ms, 4), "bound": "hbm", "unit": "GB/s",
              "peak": PEAK_HBM_GBS}
    if hb == "head.conv2.gcombine":
        hbytes = args.batch * ((H // 4) * (W // 4) * 1152 * 4 + H * W * 128 * 4 + H * W * 16)
        gfl = 2.0 * args.batch * H * W * 128 * 80   # the folded 5x5 image conv, K = 80
        hb_rec.update(kernel="up4tap_gcombine_kernel (head.conv2: tap-summed x4 bilinear "
                             "combine of the low-res tap maps + folded 5x5 image conv on "
                             "bf16x6 MFMA + IN statistics)",
                      algorithmic_bytes=hbytes,
                      achieved=round(hbytes / (hb_ms * 1e-3) / 1e9, 1),
                      frac=round(hbytes / (hb_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                      mfma_part={"flop_per_launch": gfl,
                                 "achieved_tflops": round(gfl / (hb_ms * 1e-3) / 1e12, 2),
                                 "frac_of_bf16x6_ceiling":
                                     round(gfl / (hb_ms * 1e-3) / 1e12 / arith["method_peak"], 4)})

    if rank == 0:
        rec = {
            "metric": "images/sec extract (640x480, 2048 kp)",
            "value": round(value, 3),
            "unit": "images/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen(),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "launch": launch,
            "eager_value": round(world * eager_steps * args.batch / el_eager, 3),
            "data": "synthetic (seeded uint8 480x640 images, ImageNet-normalised; seeded "
                    "random-init weights of the ResUNet-resnet50 + KeypointDet architecture)",
            "config": {"workload": "HPatches-style extraction 640x480 (configs[1]): "
                                   "PoSFeat.extract + generate_kpts_single(r=1, thr=0.9 abs, "
                                   "2048) + sample_feat_by_coord",
                       "global_batch": args.batch * world, "image": [H, W],
                       "num_pts": NUM_PTS, "parallelism": "dp%d (image-sharded)" % world},
            "roofline": {"kernel": kdesc, "label": dom,
                         "bound": "mfma", "achieved": round(achieved, 3),
                         "peak": arith["method_peak"], "unit": "TFLOP/s",
                         "frac": round(achieved / arith["method_peak"], 4),
                         "traffic": traffic,
                         "avg_launch_ms": round(kms, 4), "flop_per_launch": k_flops,
                         "arithmetic": arith["arithmetic"],
                         "fp32_mfma_peak": PEAK_FP32_MFMA_TFLOPS,
                         "frac_of_fp32_mfma_peak": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                         "note": "achieved = fp32 FLOP the launch executes / its HIP-event time "
                                 "on the engine stream; peak = the ceiling of the instruction "
                                 "mix it runs (bf16x6: dense BF16 MFMA 2500 TF / 6 products); "
                                 "frac_of_fp32_mfma_peak is the same rate against the 157.3 TF "
                                 "fp32-input MFMA peak"},
            "roofline_hbm": hb_rec,
            "head_conv2": {"ms_per_step": round(c2, 3),
                           "note": "main-stream part (low-res tap GEMM + combine); the G part "
                                   "(IN(convimg) channels) runs on the side stream",
                           "reference_equivalent_tflops":
                               round(HEAD_CONV2_FLOP_PER_IMAGE * args.batch / (c2 * 1e-3) / 1e12, 3)},
            "conv_total": {"executed_tflops": round(conv_ach, 3),
                           "frac": round(conv_ach / arith["method_peak"], 4),
                           "peak": arith["method_peak"],
                           "frac_of_fp32_mfma_peak": round(conv_ach / PEAK_FP32_MFMA_TFLOPS, 4),
                           "reference_equivalent_tflops":
                               round(CONV_FLOP_PER_IMAGE * args.batch / (conv_total * 1e-3) / 1e12, 3),
                           "ms_per_step": round(conv_total, 3),
                           "main_stream_kernels_ms_per_step": round(float(np.mean(all_ms)), 3),
                           "side_stream_kernels_ms_per_step": round(float(np.mean(side_ms)), 3),
                           "note": "main-stream launches only; the side stream (KeypointDet's "
                                   "image branch) overlaps them; frac = executed fp32-equivalent "
                                   "rate / the ceiling of the arithmetic the convs run (bf16x6: "
                                   "2500 / 6 TF)"},
        }
    if world == 1 and not args.no_secondary:
        # the two training configs' steps and their correlation losses, timed by
        # the same protocol in this process after the headline loop, so the
        # driver's N=1 run measures configs[2]/[4] too (each line's own
        # --workload run reports the full record)
        sec = {}
        for name, fn in (("corr", corr_main), ("train_kp", train_main),
                         ("train_desc", train_desc_main)):
            a2 = argparse.Namespace(**vars(args))
            a2.batch, a2.steps, a2.warmup = 8, args.secondary_steps, 3
            try:   # the headline line is printed whatever happens here
                r2 = fn(a2, world, rank, dev, emit=False)
            except Exception as e:  # noqa: BLE001
                sec[name] = {"error": "%s: %s" % (type(e).__name__, e)}
                continue
            if rank == 0:
                sec[name] = {k: r2[k] for k in ("metric", "value", "unit", "ms_per_step", "steps",
                                                "warmup")}
                sec[name]["batch_pairs"] = a2.batch
                sec[name]["roofline"] = {k: r2["roofline"].get(k) for k in
                                         ("kernel", "achieved", "peak", "unit", "frac",
                                          "arithmetic", "avg_launch_ms")}
    if rank == 0:
        if world == 1 and not args.no_secondary:
            rec["secondary_workloads"] = sec
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------
# configs[4]: keypoint-head training step (configs/train_kp.yaml, DiskLoss)


def train_main(args, world, rank, dev, emit=True):
    """One step = PoSFeat.forward over b pairs (2b images: backbone eval +
    KeypointDet), DiskLoss forward + gradient, KeypointDet backward, RCCL
    all-reduce of the 2.5 MB head gradient (world > 1), SGD update -- the
    reference's managers/trainer.py:297-356 for configs/train_kp.yaml."""
    import torch.distributed as dist
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.training import KeypointTrainStep
    b = args.batch
    engine = build_engine(world, rank, dev, train=True)
    step = KeypointTrainStep(engine, lr=1e-3)
    im1 = make_images(rank * 2 * b, b, dev)
    im2 = make_images(rank * 2 * b + b, b, dev)
    F1, F2 = [torch.from_numpy(f).to(dev) for f in synthetic_fundamental(b, H, W, 100 + rank)]
    torch.manual_seed(1234 + rank)
    for _ in range(args.warmup):
        step.step(im1, im2, F1, F2, epoch=1)
    last = {}

    def one():
        last["out"] = step.step(im1, im2, F1, F2, epoch=1)[0]
    el = timed_loop(world, args.steps, one, torch.cuda.synchronize)
    out = last["out"]
    pairs = world * args.steps * b
    # per-kernel timing of one extra step (HIP events on the engine's stream)
    engine.set_timing(2 * b, H, W, True)
    step.step(im1, im2, F1, F2, epoch=1)
    evs = engine.timing_events(2 * b, H, W, arith=True)
    engine.set_timing(2 * b, H, W, False)
    bwd_ms = sum(e[1] for e in evs if e[0].startswith("bwd"))
    fwd_ms = sum(e[1] for e in evs if e[0].startswith("conv:"))
    all_ms = sum(e[1] for e in evs)
    # dominant MFMA launch of the step (forward or backward), priced against
    # the ceiling of the arithmetic it runs
    dom = max((e for e in evs if e[2] > 0 and not e[0].startswith("side:")), key=lambda e: e[1])
    ach = dom[2] / (dom[1] * 1e-3) / 1e12
    peak, arith_name = launch_ceiling(dom[3])
    by_label = {}
    for lab, ms, _, _ in evs:
        by_label[lab] = by_label.get(lab, 0.0) + ms
    top = sorted(by_label.items(), key=lambda kv: -kv[1])[:12]
    if rank == 0:
        rec = {
            "metric": "pairs/sec keypoint-head training step (640x480, DiskLoss, SGD)",
            "value": round(pairs / el, 3), "unit": "pairs/s", "n_gpus": world,
            "ranks_seen": ranks_seen(),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded 480x640 image pairs, synthetic fundamental matrices as "
                    "datasets/megadepth.py:426-448 builds them; seeded random-init weights)",
            "config": {"workload": "configs[4]: MegaDepth-style keypoint training step "
                                   "(configs/train_kp.yaml: localheader only, DiskLoss grid 8, "
                                   "SGD lr 1e-3), %d pairs per GPU" % b,
                       "global_batch_pairs": b * world, "image": [H, W],
                       "parallelism": "dp%d (RCCL all-reduce of head grads)" % world},
            "roofline": {"kernel": dom[0], "label": dom[0],
                         "bound": "mfma", "achieved": round(ach, 3),
                         "peak": peak, "unit": "TFLOP/s",
                         "frac": round(ach / peak, 4), "traffic": None,
                         "arithmetic": arith_name,
                         "avg_launch_ms": round(dom[1], 4), "flop_per_launch": dom[2]},
            "breakdown_ms": {"forward_convs": round(fwd_ms, 3), "backward_all": round(bwd_ms, 3),
                             "engine_all": round(all_ms, 3),
                             "top_labels": {k: round(v, 3) for k, v in top}},
            "loss_last": float(out[0].item()),
        }
        if emit:
            print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return rec if rank == 0 else None


# ----------------------------------------------------------------------------
# configs[2]: descriptor training step (configs/train_desc.yaml)


def train_desc_main(args, world, rank, dev, emit=True):
    """One step = the two train-mode backbone calls of PoSFeat.forward (im1,
    im2: b images each, BatchNorm batch statistics + running update),
    Preprocess_Line2Window + EpipolarLoss_full forward and gradient, the
    backbone backward of both batches into one gradient, RCCL all-reduce of
    the 82 MB gradient (world > 1), Adam -- managers/trainer.py:293-356 for
    configs/train_desc.yaml (the keypoint head's forward feeds neither this
    loss nor any state and is not run)."""
    import torch.distributed as dist
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.training import (BackboneTrainer, DescriptorLossGrad, DESC_EPI_DEFAULTS,
                                      DESC_PRE_DEFAULTS)
    from posfeat_amd.weights import seeded_state_dicts
    b = args.batch
    bb, _ = seeded_state_dicts(0)
    # SyncBatchNorm under DDP, as PoSFeat.set_parallel converts the backbone
    tr = BackboneTrainer(bb, b, H, W, device=dev, lr=1e-4, sync_bn=world > 1)
    if world > 1:
        dist.broadcast(tr.params, src=0)
        dist.broadcast(tr.stats, src=0)
    loss = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
    im1 = make_images(rank * 2 * b, b, dev)
    im2 = make_images(rank * 2 * b + b, b, dev)
    F1, F2 = [torch.from_numpy(f).to(dev) for f in synthetic_fundamental(b, H, W, 200 + rank)]
    torch.manual_seed(4321 + rank)
    for _ in range(args.warmup):
        tr.step(im1, im2, F1, F2, loss, epoch=1)
    last = {}

    def one():
        last["out"] = tr.step(im1, im2, F1, F2, loss, epoch=1)[0]
    el = timed_loop(world, args.steps, one, torch.cuda.synchronize)
    out = last["out"]
    pairs = world * args.steps * b
    # per-kernel-class timing of one extra step (HIP events on the trainer's stream)
    tr.set_timing(True)
    tr.step(im1, im2, F1, F2, loss, epoch=1)
    cls = {k: tr.timing(k) for k in ("fwd:conv", "fwd:bn", "fwd:misc", "bwd:bn", "bwd:wgrad",
                                      "bwd:dgrad", "bwd:misc")}
    all_ms = tr.timing("")[0]
    # the conv classes per layer (labels "<class>:<layer>"), largest first
    by_layer = {}
    evs = tr.timing_events(arith=True)
    for lab, ms, fl, _ in evs:
        if lab.count(":") >= 2:
            e = by_layer.setdefault(lab, [0.0, 0.0, 0])
            e[0] += ms
            e[1] += fl
            e[2] += 1
    tr.set_timing(False)
    # the roofline names ONE launch: the step's longest MFMA conv launch,
    # priced against the ceiling of the arithmetic it runs (bf16x6 416.7,
    # fp32 MFMA 157.3)
    dom1 = max((e for e in evs if e[2] > 0 and e[0].split(":")[0] in ("fwd", "bwd")
                and e[0].split(":")[1] in ("conv", "wgrad", "dgrad")), key=lambda e: e[1])
    peak1, arith1 = launch_ceiling(dom1[3])
    ach1 = dom1[2] / (dom1[1] * 1e-3) / 1e12
    top_layers = [{"label": k, "ms": round(v[0], 3), "launches": v[2],
                   "tflops": round(v[1] / max(v[0], 1e-9) / 1e9, 1)}
                  for k, v in sorted(by_layer.items(), key=lambda kv: -kv[1][0])[:16]]
    dom = max(("fwd:conv", "bwd:wgrad", "bwd:dgrad"), key=lambda k: cls[k][0])
    d_ms, d_fl, d_n = cls[dom]
    ach = d_fl / (d_ms * 1e-3) / 1e12
    conv_ms = sum(cls[k][0] for k in ("fwd:conv", "bwd:wgrad", "bwd:dgrad"))
    conv_fl = sum(cls[k][1] for k in ("fwd:conv", "bwd:wgrad", "bwd:dgrad"))
    if rank == 0:
        rec = {
            "metric": "pairs/sec descriptor training step (640x480, Line2Window + EpipolarLoss, "
                      "Adam)",
            "value": round(pairs / el, 3), "unit": "pairs/s", "n_gpus": world,
            "ranks_seen": ranks_seen(),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded 480x640 image pairs, synthetic fundamental matrices as "
                    "datasets/megadepth.py:426-448 builds them; seeded random-init ResUNet weights)",
            "config": {"workload": "configs[2]: MegaDepth-style descriptor training step "
                                   "(configs/train_desc.yaml: backbone in train mode, "
                                   "Preprocess_Line2Window + EpipolarLoss_full, Adam 1e-4), "
                                   "%d pairs per GPU" % b,
                       "global_batch_pairs": b * world, "image": [H, W],
                       "parallelism": "dp%d (RCCL all-reduce of backbone grads%s)" % (
                           world, ", SyncBatchNorm" if world > 1 else "")},
            "roofline": {"kernel": dom1[0], "label": dom1[0],
                         "bound": "mfma", "achieved": round(ach1, 3),
                         "peak": peak1, "unit": "TFLOP/s",
                         "frac": round(ach1 / peak1, 4), "traffic": None,
                         "arithmetic": arith1,
                         "avg_launch_ms": round(dom1[1], 4), "flop_per_launch": dom1[2],
                         "note": "the step's longest MFMA conv launch (one label = one "
                                 "conv call of one layer)"},
            "dominant_class": {"class": dom, "launches": d_n, "ms": round(d_ms, 3),
                               "tflops": round(ach, 3)},
            "breakdown_ms": {k: round(v[0], 3) for k, v in cls.items()},
            "top_conv_layers": top_layers,
            "conv_total": {"ms_per_step": round(conv_ms, 3),
                           "tflops": round(conv_fl / (conv_ms * 1e-3) / 1e12, 3),
                           "backbone_kernels_ms": round(all_ms, 3)},
            "loss_last": float(out[0].item()),
        }
        if emit:
            print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return rec if rank == 0 else None


# ----------------------------------------------------------------------------
# correlation losses of the two training configs, forward + map gradients


def corr_main(args, world, rank, dev, emit=True):
    """One step = for b pairs of synthetic 480x640 local maps / score maps:
    Preprocess_Line2Window + EpipolarLoss_full and their gradient w.r.t. both
    local maps (configs[2]: training.DescriptorLossGrad), and DiskLoss with its
    gradient w.r.t. both score maps (configs[4]: KeypointTrainStep.loss_and_grad;
    flash path, S never stored).  Roofline: DiskLoss's flash LSE pass (the
    fused MFMA similarity + online logsumexp, 2 b n^2 128 FLOP, n = 4800),
    timed with HIP events on the stream it runs on."""
    import ctypes
    from posfeat_amd import _lib, ops
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.training import (DESC_EPI_DEFAULTS, DESC_PRE_DEFAULTS, DescriptorLossGrad,
                                      KeypointTrainStep)
    b = args.batch
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    # local maps: smooth random fields (as the oracle fixtures use), NHWC
    xf = torch.randn(2 * b, 128, H // 4, W // 4, device=dev, generator=g)
    xf = torch.nn.functional.avg_pool2d(xf, 3, 1, 1)
    lm = ops.nchw_to_nhwc(xf.contiguous())
    x1, x2 = lm[:b], lm[b:]
    kp = torch.rand(2 * b, 1, H, W, device=dev, generator=g) * 3
    F1, F2 = [torch.from_numpy(f).to(dev) for f in synthetic_fundamental(b, H, W, 300 + rank)]
    desc = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
    disk = KeypointTrainStep.__new__(KeypointTrainStep)
    from posfeat_amd.training import DISK_DEFAULTS
    disk.cfg, disk._ws = dict(DISK_DEFAULTS), {}
    torch.manual_seed(77 + rank)

    def one():
        desc(x1, x2, F1, F2, (H, W), (H, W), epoch=1)
        disk.loss_and_grad(kp, lm, F1, F2, epoch=1)
    for _ in range(args.warmup):
        one()
    el = timed_loop(world, args.steps, one, torch.cuda.synchronize)
    # dominant MFMA kernel: the flash LSE pass on this step's descriptors
    n = (H // 8) * (W // 8)
    fa = torch.nn.functional.normalize(torch.randn(b, n, 128, device=dev, generator=g), dim=-1)
    fb = torch.nn.functional.normalize(torch.randn(b, n, 128, device=dev, generator=g), dim=-1)
    lse = torch.empty(b, n, device=dev)
    L = _lib.lib()
    need = L.posfeat_disk_flash_lse_workspace(b, n)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)

    def lse_pass():
        _lib.check(L.posfeat_disk_flash_lse(_lib.ptr(fa), _lib.ptr(fb), b, n, 60.0, _lib.ptr(lse),
                                            _lib.ptr(ws), need, _lib.stream_ptr()))
    lse_pass()
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lse_pass()
    e1.record()
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / reps
    kfl = 2.0 * b * n * n * 128
    ach = kfl / (kms * 1e-3) / 1e12
    arith = conv_arithmetic()   # the flash passes follow the conv precision mode
    if rank == 0:
        rec = {
            "metric": "pairs/sec correlation losses + map gradients (640x480: Line2Window + "
                      "EpipolarLoss_full, DiskLoss)",
            "value": round(world * args.steps * b / el, 3), "unit": "pairs/s", "n_gpus": world,
            "ranks_seen": ranks_seen(), "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (smoothed random 128-d local maps, uniform score maps, synthetic "
                    "fundamental matrices as datasets/megadepth.py:426-448 builds them)",
            "config": {"workload": "configs[2]/[4] correlation: Preprocess_Line2Window + "
                                   "EpipolarLoss_full (train_desc.yaml) and DiskLoss "
                                   "(train_kp.yaml), forward + gradient, %d pairs per GPU" % b,
                       "global_batch_pairs": b * world, "image": [H, W],
                       "parallelism": "dp%d (pairs sharded)" % world},
            "roofline": {"kernel": "disk_flash_kernel<LSE> (DiskLoss softmax normaliser: MFMA "
                                   "similarity + online logsumexp, S never stored)",
                         "bound": "mfma", "achieved": round(ach, 3),
                         "peak": arith["method_peak"], "unit": "TFLOP/s",
                         "frac": round(ach / arith["method_peak"], 4), "traffic": None,
                         "arithmetic": arith["arithmetic"],
                         "avg_launch_ms": round(kms, 4), "flop_per_launch": kfl,
                         "timed": "one posfeat_disk_flash_lse call: two flash_split launches "
                                  "(~9 us each, the bf16 planes of both sides) + the LSE "
                                  "kernel + flash_lse_final (~5 us); rocprof's per-kernel "
                                  "time for disk_flash6_kernel<false,false> excludes the "
                                  "three small launches (DESIGN 4.1q)"},
        }
        if emit:
            print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return rec if rank == 0 else None


if __name__ == "__main__":
    main()

