"""ORACLE restatement of torchvision.models.resnet (v0.15+ semantics).

torchvision/models/resnet.py: BasicBlock / Bottleneck (stride on the 3x3,
"v1.5"), ResNet.__init__ module construction order, the init loop
(kaiming_normal_ fan_out/relu on every Conv2d, BN weight 1 / bias 0), and
forward: conv1-bn1-relu-maxpool-layer1..4-avgpool-flatten-fc.
"""
from __future__ import annotations

import enum
import os

import torch
import torch.nn as nn


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = out + identity
        return self.relu(out)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
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
        out = out + identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.dilation = 1
        self.groups = 1
        self.base_width = 64
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


class _Weights:
    def __init__(self, name, env):
        self.name, self.env = name, env

    def get_state_dict(self, progress=True, check_hash=False):
        path = os.environ.get(self.env)
        if not path:
            raise RuntimeError(f"{self.name}: pretrained weights are a network download (unavailable offline); "
                               f"set {self.env} to a local state_dict file")
        return torch.load(path, map_location="cpu", weights_only=True)

    def __repr__(self):
        return self.name


class ResNet18_Weights(enum.Enum):
    IMAGENET1K_V1 = _Weights("ResNet18_Weights.IMAGENET1K_V1", "SSIP_RESNET18_WEIGHTS")
    DEFAULT = IMAGENET1K_V1


class ResNet50_Weights(enum.Enum):
    IMAGENET1K_V1 = _Weights("ResNet50_Weights.IMAGENET1K_V1", "SSIP_RESNET50_WEIGHTS")
    DEFAULT = IMAGENET1K_V1


def _resnet(block, layers, weights, **kw):
    model = ResNet(block, layers, **kw)
    if weights is not None:
        model.load_state_dict(weights.value.get_state_dict())
    return model


def resnet18(*, weights=None, progress=True, **kw):
    return _resnet(BasicBlock, [2, 2, 2, 2], weights, **kw)


def resnet50(*, weights=None, progress=True, **kw):
    return _resnet(Bottleneck, [3, 4, 6, 3], weights, **kw)
