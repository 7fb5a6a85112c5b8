"""SyncBatchNorm semantics of the train-mode backbone (group.hip, bbtrain.hip).

The reference wraps the backbone in torch.nn.SyncBatchNorm under DDP
(networks/PoSFeat_model.py:49): with the batch split over ranks, every
BatchNorm normalises with the statistics of the WHOLE batch.  On a one-GPU box
two ranks are emulated by two threads of this process, each with its own
BackboneTrainer on half of the batch and its own stream, joined by a local
group (the same exchange points as RCCL, summed in rank order).  Checked:

* each rank's local map equals the full-batch run's rows (1e-4 of the map
  scale), and without the group it does not (the test is sensitive);
* the running statistics of both ranks equal the full-batch update;
* the sum of the ranks' gradients (what DDP's all-reduce forms, up to 1/world)
  meets the same fp64-fixture bounds as the single-rank backward
  (tests/golden/bb_grad.npz, test_bb_train._check_grads64).
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(t, ims, dms):
    """forward(im1), forward(im2), backward both into one gradient (the
    descriptor step's order, training.BackboneTrainer.step)"""
    lms = [t.forward(ims[0], 0).clone(), t.forward(ims[1], 1).clone()]
    t.backward(dms[0], 0, accumulate=False)
    t.backward(dms[1], 1, accumulate=True)
    return lms


def _run_ranks(trainers, ims, dms):
    out = [None] * len(trainers)
    err = []

    def work(r):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                out[r] = _step(trainers[r], ims[r], dms[r])
                s.synchronize()
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(len(trainers))]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not err, err
    return out


def test_syncbn_two_ranks_equal_full_batch(gpu):
    from test_bb_train import _check_grads64, _inputs
    from posfeat_amd import weights
    from posfeat_amd._lib import check, lib
    from posfeat_amd.training import BackboneTrainer
    d, im1, im2, R1, R2 = _inputs()
    b, _, H, W = im1.shape
    assert b == 2
    bb, _ = weights.seeded_state_dicts(0)
    ims = [im1.to(gpu), im2.to(gpu)]
    dms = [R.permute(0, 2, 3, 1).contiguous().to(gpu) for R in (R1, R2)]
    full = BackboneTrainer(bb, b, H, W, device=gpu)
    lm_full = _step(full, ims, dms)
    torch.cuda.synchronize()

    L = ctypes.c_void_p()
    check(lib().posfeat_local_group_create(2, 4096, ctypes.byref(L)))
    groups = []
    for r in range(2):
        g = ctypes.c_void_p()
        check(lib().posfeat_group_create_local(L, r, ctypes.byref(g)))
        groups.append(g)
    ranks = [BackboneTrainer(bb, 1, H, W, device=gpu) for _ in range(2)]
    for t, g in zip(ranks, groups):
        t.set_group(g)
    lms = _run_ranks(ranks, [[x[r:r + 1] for x in ims] for r in range(2)],
                     [[x[r:r + 1] for x in dms] for r in range(2)])
    for r in range(2):
        for s in range(2):
            scale = max(1.0, float(lm_full[s].abs().max()))
            e = float((lms[r][s][0] - lm_full[s][r]).abs().max())
            assert e <= 1e-4 * scale, "rank %d image %d map err %g" % (r, s, e)
        np.testing.assert_allclose(ranks[r].stats.cpu().numpy(), full.stats.cpu().numpy(),
                                   rtol=1e-5, atol=1e-6)
    gsum = (ranks[0].grad + ranks[1].grad).cpu().numpy()
    _check_grads64(weights.unpack_bbtrain(gsum, full.table), d)

    # control: per-rank statistics (no group) give different maps
    solo = BackboneTrainer(bb, 1, H, W, device=gpu)
    lm0 = solo.forward(ims[0][0:1], 0)
    scale = max(1.0, float(lm_full[0].abs().max()))
    assert float((lm0[0] - lm_full[0][0]).abs().max()) > 1e-2 * scale
    for g in groups:
        lib().posfeat_group_destroy(g)
    lib().posfeat_local_group_destroy(L)


def test_syncbn_unequal_batches_equal_full_batch(gpu):
    """Ranks with DIFFERENT batches (2 + 1 images: the reference Trainer's
    loader has no drop_last and my_collate drops None samples,
    managers/trainer.py:132-134): the pixel count is all-reduced with the sums
    (bbtrain.hip bn_sums_kernel), so both ranks normalise with the 3-image
    batch statistics, as torch.nn.SyncBatchNorm does.  Maps 1e-4 of scale,
    running statistics rtol 1e-5, and the summed rank gradients against the
    full-batch gradient (two fp32 summation orders of the BatchNorm-heavy
    backward: relative L2 2e-3 overall, 3e-2 of each tensor's max plus 1e-4 of
    the largest entry)."""
    from test_bb_train import _inputs
    from posfeat_amd import weights
    from posfeat_amd._lib import check, lib
    from posfeat_amd.training import BackboneTrainer
    d, im1, im2, R1, R2 = _inputs()
    _, _, H, W = im1.shape
    ims = [torch.cat([im1, im2[:1]]).to(gpu), torch.cat([im2, im1[:1]]).to(gpu)]
    dms = [torch.cat([R1, R2[:1]]).permute(0, 2, 3, 1).contiguous().to(gpu),
           torch.cat([R2, R1[:1]]).permute(0, 2, 3, 1).contiguous().to(gpu)]
    bb, _ = weights.seeded_state_dicts(0)
    full = BackboneTrainer(bb, 3, H, W, device=gpu)
    lm_full = _step(full, ims, dms)
    torch.cuda.synchronize()

    L = ctypes.c_void_p()
    check(lib().posfeat_local_group_create(2, 4096, ctypes.byref(L)))
    groups = []
    for r in range(2):
        g = ctypes.c_void_p()
        check(lib().posfeat_group_create_local(L, r, ctypes.byref(g)))
        groups.append(g)
    split = [(0, 2), (2, 3)]
    ranks = [BackboneTrainer(bb, b1 - b0, H, W, device=gpu) for b0, b1 in split]
    for t, g in zip(ranks, groups):
        t.set_group(g)
    lms = _run_ranks(ranks, [[x[b0:b1] for x in ims] for b0, b1 in split],
                     [[x[b0:b1] for x in dms] for b0, b1 in split])
    for r, (b0, b1) in enumerate(split):
        for s in range(2):
            scale = max(1.0, float(lm_full[s].abs().max()))
            e = float((lms[r][s] - lm_full[s][b0:b1]).abs().max())
            assert e <= 1e-4 * scale, "rank %d image %d map err %g" % (r, s, e)
        np.testing.assert_allclose(ranks[r].stats.cpu().numpy(), full.stats.cpu().numpy(),
                                   rtol=1e-5, atol=1e-6)
    gsum = weights.unpack_bbtrain((ranks[0].grad + ranks[1].grad).cpu().numpy(), full.table)
    gref = weights.unpack_bbtrain(full.grad.cpu().numpy(), full.table)
    num = den = 0.0
    # conv biases ahead of a BatchNorm have an exactly-zero gradient in real
    # arithmetic (fp32 noise of ~1e-5 here): a floor of 1e-4 of the largest
    # gradient entry keeps those tensors from deciding the test
    floor = 1e-4 * max(float(np.abs(v).max()) for v in gref.values())
    for k, v in gref.items():
        e = float(np.abs(gsum[k] - v).max())
        assert e <= 3e-2 * float(np.abs(v).max()) + floor, "%s: err %g of max %g" % (
            k, e, float(np.abs(v).max()))
        num += float(((gsum[k] - v) ** 2).sum())
        den += float((v ** 2).sum())
    assert num ** 0.5 <= 2e-3 * den ** 0.5
    for g in groups:
        lib().posfeat_group_destroy(g)
    lib().posfeat_local_group_destroy(L)
