"""nn.Module restatement of the torchvision ResNet-50 pieces ResUNet uses (TEST ORACLE).

``torchvision`` is a third-party dependency of the reference
(networks/DescNet.py:6-9, 25) that is absent from this image and unpinned by
the reference.  This restates its published ResNet-50 architecture (He et al.
2016; torchvision Bottleneck "v1.5": stride on the 3x3 conv, expansion 4,
BatchNorm eps 1e-5, ReLU inplace, ``downsample = Sequential(conv1x1, BN)``)
with torchvision's attribute names, so a reference ``ResUNet`` instance can be
assembled from it and load the 300-key state dict unchanged.
Only used by ``tests/golden/gen_golden.py`` to run the reference decoder code.
"""
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


def make_layer(inplanes, planes, blocks, stride):
    ds = None
    if stride != 1 or inplanes != planes * 4:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                           nn.BatchNorm2d(planes * 4))
    layers = [Bottleneck(inplanes, planes, stride, ds)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * 4, planes))
    return nn.Sequential(*layers)


class ResNet50Stem(nn.Module):
    """conv1/bn1/relu/maxpool/layer1-3 of torchvision resnet50 (attribute names kept)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = make_layer(64, 64, 3, 1)
        self.layer2 = make_layer(256, 128, 4, 2)
        self.layer3 = make_layer(512, 256, 6, 2)
