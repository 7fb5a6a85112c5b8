"""The reference Trainer's plug points under autograd (managers/trainer.py:
296-331): ``model.forward`` in train mode, the loss modules, and
``total_loss.backward()`` filling ``.grad`` of the torch modules' parameters,
then a torch optimizer step feeding the next forward.

Checked against the reference's own autograd gradients (the golden fixtures
of test_train_kp.py, test_desc_grad.py and test_bb_train.py, same tolerances)
and against the fused training APIs (KeypointTrainStep, DescriptorLossGrad)
that run the same kernels.
"""
import numpy as np
import pytest
import torch

from test_train_kp import CASES as KP_CASES, KEYS as KP_KEYS, _assert_grads, _case as _kp_case

pytestmark = pytest.mark.gpu

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


def _model(gpu):
    from posfeat_amd import networks
    from posfeat_amd.weights import seeded_state_dicts
    m = networks.PoSFeat(MODEL_CONFIG, gpu)
    bb, hd = seeded_state_dicts(0)
    m.backbone.load_state_dict(bb)
    m.localheader.load_state_dict(hd)
    return m


@pytest.mark.parametrize("tag", list(KP_CASES))
def test_kp_training_backward_vs_reference(gpu, tag):
    """train_kp: set_eval + localheader.train(), forward, DiskLoss, backward."""
    from posfeat_amd.losses import DiskLoss
    from posfeat_amd.training import DISK_DEFAULTS
    d, b, H, W, im1, im2, F1, F2, draws = _kp_case(tag)
    m = _model(gpu)
    m.set_eval()
    m.localheader.train()
    inputs = {"im1": im1, "im2": im2, "F1": F1, "F2": F2}
    outputs = m.forward(inputs)
    outputs["epoch"] = 1
    assert outputs["preds1"]["local_point"].requires_grad
    loss, comp = DiskLoss(dict(DISK_DEFAULTS))(inputs, outputs, None, draws=draws)
    np.testing.assert_allclose(float(loss), float(d[tag + "_loss"]), rtol=2e-4, atol=1e-4)
    for p in m.localheader.parameters():
        p.grad = None
    loss.backward()
    sd = dict(m.localheader.named_parameters())
    _assert_grads({k: sd[k].grad.cpu().numpy() for k in KP_KEYS}, d, tag)
    assert all(p.grad is None for p in m.backbone.parameters())


def test_kp_training_optimizer_step_feeds_next_forward(gpu):
    """torch.optim.SGD on the module parameters; the next forward packs the
    updated head (device-side) and equals an engine built from the new state."""
    from posfeat_amd.engine import ExtractionEngine
    from posfeat_amd.losses import DiskLoss
    from posfeat_amd.training import DISK_DEFAULTS, KeypointTrainStep
    d, b, H, W, im1, im2, F1, F2, draws = _kp_case("a")
    m = _model(gpu)
    m.set_eval()
    m.localheader.train()
    opt = torch.optim.SGD(m.localheader.parameters(), lr=0.5)
    inputs = {"im1": im1, "im2": im2, "F1": F1, "F2": F2}
    outputs = m.forward(inputs)
    outputs["epoch"] = 1
    loss, _ = DiskLoss(dict(DISK_DEFAULTS))(inputs, outputs, None, draws=draws)
    opt.zero_grad()
    loss.backward()
    opt.step()
    # the fused step with the same draws and lr gives the same new head
    from posfeat_amd.weights import seeded_state_dicts
    bb, hd = seeded_state_dicts(0)
    eng = ExtractionEngine(bb, hd, device=gpu, train=True)
    KeypointTrainStep(eng, lr=0.5).step(im1.to(gpu), im2.to(gpu), F1, F2, epoch=1, draws=draws)
    from posfeat_amd import _lib, weights
    fused = weights.unpack_head(eng.head_weights().cpu().numpy(), _lib.model_specs())
    for k, p in m.localheader.state_dict().items():
        np.testing.assert_allclose(p.cpu().numpy().reshape(-1), fused[k].reshape(-1),
                                   rtol=1e-6, atol=1e-7, err_msg=k)
    with torch.no_grad():
        out2 = m.forward(inputs)
    fresh = ExtractionEngine(m.backbone.state_dict(), m.localheader.state_dict(), device=gpu)
    ref = fresh.run(torch.cat([im1, im2]).to(gpu))
    got = torch.cat([out2["preds1"]["local_point"], out2["preds2"]["local_point"]])
    scale = max(1.0, float(ref["local_point"].abs().max()))
    assert float((got - ref["local_point"]).abs().max()) <= 1e-5 * scale
    outputs = m.forward(inputs)     # grad mode again: the train engine re-synced
    got = torch.cat([outputs["preds1"]["local_point"], outputs["preds2"]["local_point"]]).detach()
    assert float((got - ref["local_point"]).abs().max()) <= 1e-5 * scale


def test_desc_losses_backward_vs_fused_and_reference(gpu):
    """Preprocess_Line2Window + EpipolarLoss_full on maps that require grad:
    loss.backward() gives DescriptorLossGrad's dL/d maps, and the reference's."""
    from test_desc_grad import EPI_CFG, PRE_CFG, _case as _desc_case, _close, _gpu
    from posfeat_amd.losses import EpipolarLoss_full, Preprocess_Line2Window
    d, b, H, W, xf1, xf2, F1, F2, draws = _desc_case("m")
    x1 = xf1.to(gpu).requires_grad_()
    x2 = xf2.to(gpu).requires_grad_()
    inputs = {"im1": torch.zeros(b, 3, H, W, device=gpu), "im2": torch.zeros(b, 3, H, W, device=gpu),
              "F1": F1, "F2": F2}
    outputs = {"preds1": {"local_map": x1}, "preds2": {"local_map": x2}, "epoch": 0}
    sel1, sel2, r1, r2 = draws
    processed = Preprocess_Line2Window(PRE_CFG)(inputs, outputs,
                                                draws=(sel1.int(), sel2.int(), r1, r2))
    loss, comp = EpipolarLoss_full(EPI_CFG)(inputs, outputs, processed)
    (2.0 * loss).backward()
    _, _, out, dx1, dx2, _ = _gpu(gpu, "m")
    assert float(loss) == float(out[0])
    np.testing.assert_array_equal(x1.grad.cpu().numpy(), 2.0 * dx1.numpy())
    np.testing.assert_array_equal(x2.grad.cpu().numpy(), 2.0 * dx2.numpy())
    _close(x1.grad.cpu().numpy() / 2, d["m_dxf1"], 1e-3, "dxf1")


def test_backbone_training_backward_vs_reference(gpu):
    """train_desc: set_eval + backbone.train(), forward (two train-mode ResUNet
    calls), loss = sum(local_map1 * R1) + sum(local_map2 * R2), backward: the
    gradient fixture of test_bb_train.py (reference ResUNet, fp64), and the
    running statistics / num_batches_tracked written back into the buffers."""
    from test_bb_train import _check_grads64, _inputs
    from posfeat_amd.training import BackboneTrainer
    from posfeat_amd.weights import seeded_state_dicts
    d, im1, im2, R1, R2 = _inputs()
    m = _model(gpu)
    m.set_eval()
    m.backbone.train()
    outputs = m.forward({"im1": im1, "im2": im2})
    lm1, lm2 = outputs["preds1"]["local_map"], outputs["preds2"]["local_map"]
    loss = (lm1 * R1.to(gpu)).sum() + (lm2 * R2.to(gpu)).sum()
    loss.backward()
    got = {k: (p.grad.cpu().numpy() if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
           for k, p in m.backbone.named_parameters()}
    assert m.backbone.conv_coarse.conv.weight.grad is None
    _check_grads64(got, d)
    # running statistics: the same as the fused trainer's after its two forwards
    bb, _ = seeded_state_dicts(0)
    tr = BackboneTrainer(bb, im1.shape[0], im1.shape[2], im1.shape[3], device=gpu)
    tr.forward(im1.to(gpu), 0)
    tr.forward(im2.to(gpu), 1)
    sd = tr.state_dict()
    for k, v in m.backbone.state_dict().items():
        if "running" in k or "num_batches" in k:
            np.testing.assert_array_equal(v.cpu().numpy().reshape(-1),
                                          np.asarray(sd[k]).reshape(-1), err_msg=k)
