"""torch-CPU restatement of the keypoint-head training step (TEST ORACLE ONLY).

Test infrastructure: imported by tests/ and tools/ only, never by posfeat_amd/.

Follows managers/trainer.py:286-356 with configs/train_kp.yaml (only
``localheader`` trains, SGD lr 1e-3, DiskLoss): PoSFeat.forward
(PoSFeat_model.py:136-147; backbone maps detached, 97-102) ->
DiskLoss.forward (losses/kploss.py:132-197, constant_reward, cor_detach,
match_grad False) -> autograd backward -> SGD step.  The DiskLoss random
draws (Categorical proposals and Bernoulli acceptances, kploss.py:20-35) are
explicit inputs so the GPU path can replay them.
"""
import torch
import torch.nn.functional as F

from .correlation_ref import disk_point_logp, homogenize, normalize_coords, sample_feat
from .model_ref import keypointdet_forward, resunet_forward


def disk_loss_autograd(kp1, kp2, xf1, xf2, F1, F2, prop1, prop2, acc1, acc2, temperature=60.0,
                       g=8, reward_thr=2.0, good=1.0, bad=-0.25, kp_penalty=-0.001):
    """DiskLoss.forward (kploss.py:132-197) keeping the graph to kp1/kp2:
    sample_p is detached (cor_detach, 168-171) and the match costs carry no
    gradient (match_grad False, 155-159)."""
    b, _, h, w = kp1.shape
    c1, logp1 = disk_point_logp(kp1, g, prop1, acc1)
    c2, logp2 = disk_point_logp(kp2, g, prop2, acc2)
    with torch.no_grad():
        f1 = sample_feat(xf1, normalize_coords(c1, h, w), True)
        f2 = sample_feat(xf2, normalize_coords(c2, h, w), True)
        aff = -temperature * (1 - f1 @ f2.transpose(1, 2))
        lrow = torch.log_softmax(aff, dim=2)
        lcol = torch.log_softmax(aff, dim=1)
        dense_p = lrow.exp() * lcol.exp()
        dense_logp = lrow + lcol
        l1 = F1.bmm(homogenize(c1).transpose(1, 2))
        l1 = l1 / torch.clamp(torch.norm(l1[:, :2, :], p=2, dim=1, keepdim=True), min=1e-8)
        d1 = torch.abs(l1.transpose(1, 2) @ homogenize(c2).transpose(1, 2))
        l2 = F2.bmm(homogenize(c2).transpose(1, 2))
        l2 = l2 / torch.clamp(torch.norm(l2[:, :2, :], p=2, dim=1, keepdim=True), min=1e-8)
        d2 = torch.abs(l2.transpose(1, 2) @ homogenize(c1).transpose(1, 2)).transpose(1, 2)
        good_m = (d1 < reward_thr) & (d2 < reward_thr)
        reward = good * good_m + bad * (~good_m)
    kps_logp = logp1.reshape(b, 1, -1).transpose(1, 2) + logp2.reshape(b, 1, -1)
    plogp = dense_p * (dense_logp + kps_logp)
    am = acc1.reshape(b, 1, -1).transpose(1, 2) * acc2.reshape(b, 1, -1)
    reinforce = (reward[am] * plogp[am]).sum()
    penalty = kp_penalty * (logp1[acc1].sum() + logp2[acc2].sum())
    return -reinforce - penalty


def head_step(bb_sd, hd_sd, im1, im2, F1, F2, draws, temperature=60.0, lr=1e-3):
    """One config-5 step.  Returns (loss, grads{key: tensor}, new head sd,
    local_point maps).  ``draws`` = (prop1, prop2, acc1, acc2) shaped like
    kploss.point_sample's outputs ([b,1,h/8,w/8])."""
    params = {k: v.clone().float().requires_grad_(True) for k, v in hd_sd.items()}
    lps, lmaps = [], []
    for im in (im1, im2):
        with torch.no_grad():
            feat = resunet_forward(bb_sd, im)
        local_input = torch.cat([feat["local_map"], feat["local_map_small"]], 1).detach()
        lps.append(keypointdet_forward(params, local_input, im))
        lmaps.append(feat["local_map"])
    prop1, prop2, acc1, acc2 = draws
    loss = disk_loss_autograd(lps[0], lps[1], lmaps[0], lmaps[1], F1, F2, prop1, prop2, acc1, acc2,
                              temperature)
    grads = torch.autograd.grad(loss, [params[k] for k in hd_sd])
    grads = {k: g.detach() for k, g in zip(hd_sd, grads)}
    new = {k: (hd_sd[k].float() - lr * grads[k]) for k in hd_sd}
    return loss.detach(), grads, new, [lp.detach() for lp in lps]
