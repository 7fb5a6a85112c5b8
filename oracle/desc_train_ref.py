"""torch-CPU restatement of the descriptor-training loss gradient (TEST ORACLE ONLY).

Test infrastructure: imported by tests/ and tools/ only, never by posfeat_amd/.

configs/train_desc.yaml (weight_grid 0, weight_window 1, use_std_as_weight):
Preprocess_Line2Window (losses/preprocess.py:27-121; the line search runs
under no_grad, preprocess_utils.py:661) + EpipolarLoss_full
(losses/epipolarloss.py:38-101; the std weights are detached, 25-36), with
autograd giving dL/d local_map for both images -- what loss.backward()
(managers/trainer.py:331) sends into the backbone.
"""
import torch
import torch.nn.functional as F

from .correlation_ref import (_epipolar_cost, denormalize_coords, epipolar_line_search,
                              get_endpoints, grid_points, sample_feat, window_expectation)


def desc_loss_grad(xf1, xf2, F1, F2, hw1, hw2, sel1, sel2, rand1, rand2, temperature=60.0,
                   grid_size=16, window_size=0.1, line_step=100, win_cost_thr=0.1,
                   centers=None, weights=None):
    """Returns (loss, dxf1, dxf2, (l1, l2)).  ``centers`` = (l1, l2) window
    centres to use instead of this function's own line search (so a test can
    share the GPU's arg-max on near-ties); their validity is re-derived as the
    reference does (endpoints valid & centre inside the image).  ``weights`` =
    the two detached per-point loss weights (see loss_weights) to use as given."""
    (h1i, w1i), (h2i, w2i) = hw1, hw2
    xf1 = xf1.detach().clone().requires_grad_(True)
    xf2 = xf2.detach().clone().requires_grad_(True)
    c1n = grid_points(sel1, h1i, w1i, grid_size)
    c2n = grid_points(sel2, h2i, w2i, grid_size)
    coord1 = denormalize_coords(c1n, h1i, w1i)
    coord2 = denormalize_coords(c2n, h2i, w2i)
    f1 = sample_feat(xf1, c1n, True)
    f2 = sample_feat(xf2, c2n, True)
    fm2 = temperature * F.normalize(xf2, p=2.0, dim=1)
    fm1 = temperature * F.normalize(xf1, p=2.0, dim=1)
    with torch.no_grad():
        l1, _, v1, _ = epipolar_line_search(coord1, F1, f1, fm2, h2i, w2i, rand1, line_step,
                                            window_size)
        l2, _, v2, _ = epipolar_line_search(coord2, F2, f2, fm1, h1i, w1i, rand2, line_step,
                                            window_size)
        if centers is not None:
            l1, l2 = centers

            def border(e):
                return (e[..., 0] >= -1) & (e[..., 0] <= 1) & (e[..., 1] >= -1) & (e[..., 1] <= 1)
            v1 = get_endpoints(coord1, F1, h2i, w2i)[2] & border(l1)
            v2 = get_endpoints(coord2, F2, h1i, w1i)[2] & border(l2)
    w1n, _, w1s = window_expectation(f1, fm2, l1, window_size)
    w2n, _, w2s = window_expectation(f2, fm1, l2, window_size)
    short = min(h1i, w1i)
    loss = 0.0
    for i, (cq, wn, sd, Fm, v, (hh, ww)) in enumerate(((coord1, w1n, w1s, F1, v1, (h2i, w2i)),
                                                      (coord2, w2n, w2s, F2, v2, (h1i, w1i)))):
        cost = _epipolar_cost(cq, denormalize_coords(wn, hh, ww), Fm)
        if weights is not None:
            wgt = weights[i]
        else:
            wgt = loss_weights(cq, denormalize_coords(wn, hh, ww).detach(), sd.detach(), v, Fm,
                               short, win_cost_thr)
        loss = loss + (wgt * cost).mean()
    g1, g2 = torch.autograd.grad(loss, [xf1, xf2])
    return loss.detach(), g1, g2, (l1, l2)


def loss_weights(coord, wpx, std, valid, Fm, short, win_cost_thr=0.1):
    """EpipolarLoss_full.set_weight for the window branch (epipolarloss.py:25-36,
    64-85): (1/std)/mean(1/std) * mask / (mean(...) + 1e-8), detached; mask =
    cost < short * win_cost_thr & valid.  Takes the forward's outputs, so a test
    can hand the oracle the exact weights the GPU path used (a point at the
    mask threshold, or with an fp32-cancelled std, otherwise flips between them)."""
    with torch.no_grad():
        cost = _epipolar_cost(coord, wpx, Fm)
        mask = (cost < short * win_cost_thr) & valid
        inv = 1 / std.clamp(min=1e-10)
        wgt = (inv / torch.mean(inv)) * mask.float()
        return wgt / (torch.mean(wgt) + 1e-8)
