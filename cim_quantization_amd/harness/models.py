"""CIFAR ResNets (He et al., option-A identity shortcuts) with the module names and parameter
layout of the reference's models/cifar10/resnet.py (conv1/bn1, layer{1,2,3}.{i}.conv{1,2}/bn{1,2},
linear), so checkpoints and state_dict keys carry over unchanged.  ``pretrained`` weights are
fetched from the network by the reference (resnet.py:127-128); here they come from a local file
(``pretrained_location`` in the prototxt) or not at all.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["resnet20", "resnet32", "resnet44", "resnet56", "resnet110", "resnet1202", "ResNet"]


class PadShortcut(nn.Module):
    """Option A: stride-2 subsampling plus zero channels on both sides (no parameters)."""

    def __init__(self, extra):
        super().__init__()
        self.extra = extra

    def forward(self, x):
        return F.pad(x[:, :, ::2, ::2], (0, 0, 0, 0, self.extra, self.extra))


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = PadShortcut(cout // 4) if (stride != 1 or cin != cout) else nn.Sequential()

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + self.shortcut(x))


class ResNet(nn.Module):
    def __init__(self, blocks_per_stage, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 16, 3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(16)
        cin = 16
        stages = []
        for width, stride in ((16, 1), (32, 2), (64, 2)):
            blocks = []
            for i in range(blocks_per_stage):
                blocks.append(BasicBlock(cin, width, stride if i == 0 else 1))
                cin = width
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3 = stages
        self.linear = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer3(self.layer2(self.layer1(y)))
        y = F.avg_pool2d(y, y.shape[3]).flatten(1)
        return self.linear(y)


def _make(n, pretrained=False, pretrained_location=None):
    model = ResNet(n)
    if pretrained:
        if not pretrained_location:
            raise RuntimeError("pretrained weights need a local file (pretrained_location); there is no download")
        sd = torch.load(pretrained_location, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd)
        model.load_state_dict({k[7:] if k.startswith("module.") else k: v for k, v in sd.items()})
    return model


def resnet20(pretrained=False, **kw):
    return _make(3, pretrained, **kw)


def resnet32(pretrained=False, **kw):
    return _make(5, pretrained, **kw)


def resnet44(pretrained=False, **kw):
    return _make(7, pretrained, **kw)


def resnet56(pretrained=False, **kw):
    return _make(9, pretrained, **kw)


def resnet110(pretrained=False, **kw):
    return _make(18, pretrained, **kw)


def resnet1202(pretrained=False, **kw):
    return _make(200, pretrained, **kw)
