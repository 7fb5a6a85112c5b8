"""One rank of tests/test_gpu_multirank.py's descriptor-training step (not a
test module).  Rank / world / device come from the torchrun environment
(RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT); the process group's
backend from POSFEAT_DIST_BACKEND (parallel.dist_backend: gloo when two ranks
share one device).

The step goes through the reference Trainer's plug points
(/root/reference/managers/trainer.py:128-173, 293-331): PoSFeat in train
mode (set_eval + backbone.train()), ``set_parallel`` at world > 1 (weights
broadcast from rank 0, SyncBatchNorm statistics over the ranks, gradients
averaged over the ranks as DDP does), ``forward`` on this rank's slice of the
batch, a loss, ``loss.backward()``.  Writes this rank's backbone gradients,
running statistics and local maps to an npz.

usage: python tests/mr_worker.py fixture|bench <out.npz, "{rank}" -> RANK>
  fixture: tests/test_bb_train.py's case (2 image pairs, 128x160), loss =
           sum(local_map * R) as the fp64 golden fixture was made;
  bench:   8 pairs at 480x640 (configs[2]'s bench shape), loss = the mean over
           this rank's pairs of sum(local_map * R) -- DDP's rank-mean of
           per-rank means is then the world-1 mean over all 8 pairs.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

MODEL_CONFIG = {
    "backbone": "ResUNet",
    "backbone_config": {"encoder": "resnet50", "pretrained": True, "coarse_out_ch": 128,
                        "fine_out_ch": 128},
    "localheader": "KeypointDet",
    "localheader_config": {"in_channels": 192, "prior": "identity", "act": "Softplus"},
    "align_local_grad": False,
    "local_input_elements": ["local_map", "local_map_small"],
    "local_with_img": True,
}


def bench_inputs(b=8, h=480, w=640):
    from posfeat_amd.weights import seeded_image
    im1 = torch.from_numpy(np.stack([seeded_image(60 + i, h, w) for i in range(b)]))
    im2 = torch.from_numpy(np.stack([seeded_image(80 + i, h, w) for i in range(b)]))
    rs = np.random.RandomState(5)
    R1 = torch.from_numpy(rs.randn(b, 128, h // 4, w // 4).astype(np.float32))
    R2 = torch.from_numpy(rs.randn(b, 128, h // 4, w // 4).astype(np.float32))
    return im1, im2, R1, R2


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    case, out = sys.argv[1], sys.argv[2].format(rank=rank)
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dev = torch.device("cuda", torch.cuda.current_device())
    if world > 1:
        from posfeat_amd.parallel import dist_backend
        dist.init_process_group(backend=dist_backend())
    from posfeat_amd import networks
    from posfeat_amd.weights import seeded_state_dicts
    if case == "fixture":
        from test_bb_train import _inputs
        _, im1, im2, R1, R2 = _inputs()
    else:
        im1, im2, R1, R2 = bench_inputs()
    b = im1.shape[0] // world
    sl = slice(rank * b, (rank + 1) * b)
    m = networks.PoSFeat(MODEL_CONFIG, dev)
    bb, hd = seeded_state_dicts(0)
    m.backbone.load_state_dict(bb)
    m.localheader.load_state_dict(hd)
    m.set_eval()
    m.backbone.train()
    if world > 1:
        m.set_parallel(int(os.environ.get("LOCAL_RANK", "0")))
    outputs = m.forward({"im1": im1[sl].clone(), "im2": im2[sl].clone()})
    lm1, lm2 = outputs["preds1"]["local_map"], outputs["preds2"]["local_map"]
    scale = 1.0 if case == "fixture" else 1.0 / b
    loss = ((lm1 * R1[sl].to(dev)).sum() + (lm2 * R2[sl].to(dev)).sum()) * scale
    loss.backward()
    res = {"lm1": lm1.detach().cpu().numpy(), "lm2": lm2.detach().cpu().numpy(),
           "loss": np.float64(loss.item()), "world": np.int64(world), "rank": np.int64(rank)}
    for k, p in m.backbone.named_parameters():
        if p.grad is not None:
            res["g/" + k] = p.grad.cpu().numpy()
    for k, v in m.backbone.state_dict().items():
        if "running" in k or "num_batches" in k:
            res["s/" + k] = v.cpu().numpy()
    np.savez(out, **res)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
