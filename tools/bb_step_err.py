"""Per-tensor error of one full config-3 training step against the fp64
oracle (tests/test_bb_train.py::test_gpu_desc_train_step_vs_oracle, printing
instead of asserting).  usage: [POSFEAT_BF6X=0] python tools/bb_step_err.py [precision]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    from posfeat_amd._lib import lib
    if len(sys.argv) > 1:
        lib().posfeat_set_conv_precision(int(sys.argv[1]))
    import test_bb_train as T
    from oracle.desc_train_ref import desc_loss_grad, loss_weights
    from oracle.model_ref import resunet_forward
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.training import DescriptorLossGrad
    from posfeat_amd.weights import seeded_state_dicts
    from test_desc_grad import EPI_CFG, PRE_CFG
    gpu = "cuda:0"
    d, im1, im2, _, _ = T._inputs()
    b, H, W, seed = T.CASE
    F1, F2 = [torch.from_numpy(f) for f in synthetic_fundamental(b, H, W, seed)]
    n = (H // 16) * (W // 16)
    g = torch.Generator().manual_seed(seed)
    hg, wg = H // 16, W // 16
    draws = (torch.randint(0, 256, (b, hg, wg), generator=g),
             torch.randint(0, 256, (b, hg, wg), generator=g),
             torch.rand(b, n, 2, generator=g), torch.rand(b, n, 2, generator=g))
    tr = T._trainer(gpu, lr=1e-3)
    out, res = tr.step(im1.to(gpu), im2.to(gpu), F1, F2, DescriptorLossGrad(PRE_CFG, EPI_CFG),
                       epoch=0, draws=(draws[0].int(), draws[1].int(), draws[2], draws[3]),
                       update=False)
    torch.cuda.synchronize()
    res = {k: v.cpu() for k, v in res.items()}
    bb, _ = seeded_state_dicts(0)
    sd = {k: (v.clone().double() if v.is_floating_point() else v.clone()) for k, v in bb.items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items()
              if not ("running" in k or "num_batches" in k)}
    x1 = resunet_forward(sd, im1.double(), train=True)["local_map"]
    x2 = resunet_forward(sd, im2.double(), train=True)["local_map"]
    wts = [loss_weights(res["coord%d" % i], res["w%d" % i], res["w%d_std" % i],
                        res["valid%d" % i].bool(), Fm, min(H, W)) for i, Fm in ((1, F1), (2, F2))]
    loss, g1, g2, _ = desc_loss_grad(x1.detach().float(), x2.detach().float(), F1, F2, (H, W),
                                     (H, W), *draws, centers=(res["l1_exp_n"], res["l2_exp_n"]),
                                     weights=wts)
    print("loss gpu %.6f oracle %.6f" % (float(out[0]), float(loss)))
    keys = [k for k in params if "stat_" + k in d.files and not k.endswith("conv.bias")]
    grads = torch.autograd.grad([x1, x2], [params[k] for k in keys],
                                grad_outputs=[g1.double(), g2.double()])
    got = tr.grad_dict()
    rows, num, den = [], 0.0, 0.0
    for k, gr in zip(keys, grads):
        ref = gr.numpy()
        gk = np.asarray(got[k], np.float64).reshape(ref.shape)
        rows.append((np.abs(gk - ref).max() / max(np.abs(ref).max(), 1e-12), k))
        num += float(((gk - ref) ** 2).sum())
        den += float((ref ** 2).sum())
    rows.sort(reverse=True)
    for e, k in rows[:8]:
        print("%-40s %.4f" % (k, e))
    print("relative L2 over all: %.5f" % np.sqrt(num / den))


if __name__ == "__main__":
    main()
