"""Run-to-run bit identity of the hot-path kernels on identical inputs.

Round 4 found a kernel (the first packed-FMA form of up4tap_gcombine_kernel)
whose results differed between identical launches in lanes 48-63 of a wave
(DESIGN.md 4.1r).  tools/isa_check.py now fails a build holding that
instruction form (v_pk_fma_f32 whose low result reads the high dword of its
own destination) and REPORTS the same in-place low<-high read on
v_pk_add_f32 / v_pk_mov_b32, which the compiler emits in ocml's log1pf
(softplus_norm4_kernel, disk_point_kernel) and in 64-bit pair copies
(disk_flash6_kernel, epi_loss_bwd_kernel, gfuse_ring_kernel).  These tests are
the empirical half: every kernel that holds a reported instance runs many
times on the same inputs and must give the same bits each time.

* extraction forward at the benchmarked size class (B = 8, 480x640: every
  extraction kernel, softplus_norm4 and gfuse_ring included), 12 repeats;
* the correlation losses and their map gradients (Line2Window +
  EpipolarLoss_full backward, epi_loss_bwd; DiskLoss flash passes + score-map
  gradient, disk_point / disk_flash6), same draws, 12 repeats.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, W = 480, 640
NREP = 12


def test_extraction_forward_repeats_bit_identical(gpu):
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.weights import seeded_image, seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device=gpu)
    imgs = torch.from_numpy(np.stack([seeded_image(300 + i, H, W) for i in range(8)])).to(gpu)
    ref = None
    try:
        for k in range(NREP):
            out = eng.run(imgs, outputs=("local_map", "global_map", "global_feat"))
            cur = {n: out[n].clone() for n in ("local_point", "local_map", "global_feat")}
            if ref is None:
                ref = cur
                continue
            for n in ref:
                bad = (cur[n] != ref[n]).sum().item()
                assert bad == 0, "repeat %d: %s differs in %d elements" % (k, n, bad)
    finally:
        eng.close()


def test_correlation_losses_repeat_bit_identical(gpu):
    from posfeat_amd import ops
    from posfeat_amd.correlation import synthetic_fundamental
    from posfeat_amd.training import (DESC_EPI_DEFAULTS, DESC_PRE_DEFAULTS, DISK_DEFAULTS,
                                      DescriptorLossGrad, KeypointTrainStep)
    b = 4
    g = torch.Generator(device=gpu).manual_seed(5)
    xf = torch.nn.functional.avg_pool2d(torch.randn(2 * b, 128, H // 4, W // 4, device=gpu,
                                                    generator=g), 3, 1, 1)
    lm = ops.nchw_to_nhwc(xf.contiguous())
    kp = torch.rand(2 * b, 1, H, W, device=gpu, generator=g) * 3
    F1, F2 = [torch.from_numpy(f).to(gpu) for f in synthetic_fundamental(b, H, W, 7)]
    n1 = (H // 16) * (W // 16)
    torch.manual_seed(11)
    ddraws = [torch.randint(0, 256, (b, n1), dtype=torch.int32),
              torch.randint(0, 256, (b, n1), dtype=torch.int32),
              torch.rand(b, n1, 2), torch.rand(b, n1, 2)]
    nk = (H // 8) * (W // 8)
    kdraws = [torch.randint(0, 64, (b, nk), dtype=torch.int32),
              torch.randint(0, 64, (b, nk), dtype=torch.int32),
              torch.rand(b, nk) < 0.5, torch.rand(b, nk) < 0.5]
    desc = DescriptorLossGrad(DESC_PRE_DEFAULTS, DESC_EPI_DEFAULTS)
    disk = KeypointTrainStep.__new__(KeypointTrainStep)
    disk.cfg, disk._ws = dict(DISK_DEFAULTS), {}
    ref = None
    for k in range(NREP):
        out, dx1, dx2, _ = desc(lm[:b], lm[b:], F1, F2, (H, W), (H, W), epoch=1, draws=ddraws)
        dout, dkp = disk.loss_and_grad(kp, lm, F1, F2, epoch=1, draws=kdraws)
        cur = {"epi": out.clone(), "dx1": dx1.clone(), "dx2": dx2.clone(), "disk": dout.clone(),
               "dkp": dkp.clone()}
        if ref is None:
            ref = cur
            assert all(torch.isfinite(v).all().item() for v in cur.values())
            continue
        for n in ref:
            bad = (cur[n] != ref[n]).sum().item()
            assert bad == 0, "repeat %d: %s differs in %d elements" % (k, n, bad)
