"""torch-CPU fp32 restatement of the PoSFeat extraction network (TEST ORACLE).

Functional form over a state dict; every block cites the reference.  The
ResNet-50 encoder is the third-party ``torchvision.models.resnet50``
(networks/DescNet.py:25), which is not installed in this image and is not
pinned by the reference (no requirements file).  It is restated here from
its published architecture (He et al. 2016, torchvision "v1.5" Bottleneck:
stride on the 3x3 conv, expansion 4, BN eps 1e-5); the parameter names match
the torchvision layout (300-key state dict).
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def _bn(x, sd, p, train=False):
    """BatchNorm2d; train=True: batch statistics and the in-place running-stat
    update of nn.BatchNorm2d.train() (momentum 0.1)."""
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], training=train, momentum=0.1,
                        eps=BN_EPS)


def _bottleneck(x, sd, p, stride, has_ds, train=False):
    """torchvision Bottleneck.forward (restated)."""
    idt = x
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1", train))
    out = F.relu(_bn(F.conv2d(out, sd[p + ".conv2.weight"], stride=stride, padding=1), sd,
                     p + ".bn2", train))
    out = _bn(F.conv2d(out, sd[p + ".conv3.weight"]), sd, p + ".bn3", train)
    if has_ds:
        idt = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd,
                  p + ".downsample.1", train)
    return F.relu(out + idt)


def _conv_bn_elu(x, sd, p, k, train=False):
    """DescNet.conv.forward: elu(bn(conv(x))) with padding (k-1)//2 (DescNet.py:167-179)."""
    y = F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], padding=(k - 1) // 2)
    return F.elu(_bn(y, sd, p + ".bn", train))


def _upconv(x, sd, p, train=False):
    """DescNet.upconv.forward: bilinear x2 align_corners=True then conv (DescNet.py:182-190)."""
    x = F.interpolate(x, scale_factor=2, align_corners=True, mode="bilinear")
    return _conv_bn_elu(x, sd, p + ".conv", 3, train)


def _skipconnect(x1, x2):
    """DescNet.ResUNet.skipconnect: pad x1 to x2, cat([x2, x1]) (DescNet.py:50-62)."""
    dy = x2.size(2) - x1.size(2)
    dx = x2.size(3) - x1.size(3)
    x1 = F.pad(x1, (dx // 2, dx - dx // 2, dy // 2, dy - dy // 2))
    return torch.cat([x2, x1], dim=1)


def resunet_forward(sd, x, train=False):
    """ResUNet.forward (DescNet.py:64-84) with the ResNet-50 encoder restated.
    train=True: BatchNorm in training mode (backbone.train(), trainer.py:293-296);
    the running statistics in ``sd`` are updated in place."""
    x = F.relu(_bn(F.conv2d(x, sd["firstconv.weight"], stride=2, padding=3), sd, "firstbn", train))
    x_first = F.max_pool2d(x, 3, 2, 1)
    h = x_first
    feats = []
    for lname, blocks, stride in (("layer1", 3, 1), ("layer2", 4, 2), ("layer3", 6, 2)):
        for bi in range(blocks):
            h = _bottleneck(h, sd, "%s.%d" % (lname, bi), stride if bi == 0 else 1, bi == 0, train)
        feats.append(h)
    x1, x2, x3 = feats
    x_coarse = _conv_bn_elu(x3, sd, "conv_coarse", 1, train)
    x = _upconv(x3, sd, "upconv3", train)
    x = _skipconnect(x2, x)
    x = _conv_bn_elu(x, sd, "iconv3", 3, train)
    x = _upconv(x, sd, "upconv2", train)
    x = _skipconnect(x1, x)
    x = _conv_bn_elu(x, sd, "iconv2", 3, train)
    x_fine = _conv_bn_elu(x, sd, "conv_fine", 1, train)
    return {"global_map": x_coarse, "local_map": x_fine, "local_map_small": x_first}


def keypointdet_forward(sd, fine_map, img):
    """KeypointDet.forward with prior='identity', act='Softplus' (DeteNet.py:102-121).

    The identity prior is ``ones.mean(1)`` so ``x_pf*fine_map == fine_map`` and
    the final rescale multiplies by exactly 1.0 (DeteNet.py:97-99, 118-119).
    """
    a = sd["relu.weight"]
    x = F.prelu(F.instance_norm(F.conv2d(fine_map, sd["conv1.weight"], sd["conv1.bias"], padding=1)), a)
    x = F.interpolate(x, img.shape[2:], align_corners=False, mode="bilinear")
    im = F.instance_norm(F.conv2d(img, sd["convimg.weight"], sd["convimg.bias"], padding=1))
    x = torch.cat([x, im], dim=1)
    x = F.prelu(F.instance_norm(F.conv2d(x, sd["conv2.weight"], sd["conv2.bias"], padding=1)), a)
    score = F.softplus(F.instance_norm(F.conv2d(x, sd["conv3.weight"], sd["conv3.bias"])))
    return score


@torch.no_grad()
def posfeat_extract(bb_sd, hd_sd, img):
    """PoSFeat.extract (networks/PoSFeat_model.py:91-134) for the effective
    extraction config (local_input_elements=[local_map, local_map_small],
    align_local_grad=False, local_with_img=True; train_desc.yaml:29-31)."""
    feat = resunet_forward(bb_sd, img)
    b, c, h, w = feat["global_map"].shape
    g_map = torch.ones(b, 1, h, w, dtype=img.dtype)
    local_input = torch.cat([feat["local_map"], feat["local_map_small"]], dim=1)
    l_map = keypointdet_forward(hd_sd, local_input, img)
    local_thr = torch.zeros_like(l_map)
    g_desc = F.normalize(g_map * feat["global_map"], p=2, dim=1).mean([2, 3])
    return {"local_map": feat["local_map"], "global_map": feat["global_map"],
            "global_feat": g_desc, "local_point": l_map, "local_thr": local_thr,
            "global_point": g_map, "local_map_small": feat["local_map_small"]}
