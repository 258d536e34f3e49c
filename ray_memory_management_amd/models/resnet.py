"""ResNet-18/34/50/101/152 for the Train benchmarks (the reference's AIR benchmarks train
torchvision ResNets: release/air_tests/air_benchmarks/workloads/pytorch_training_e2e.py,
torch_benchmark.py). torchvision is not part of this stack, so the architecture (He et al. 2015,
v1.5: stride on the 3x3 conv of the bottleneck) is defined here.

MI355X layout: build with ``memory_format=torch.channels_last`` so MIOpen runs NHWC implicit-GEMM
(MFMA) kernels without layout transposes; train under bf16 autocast. ``zero_init_residual`` zeroes
the last BN gamma of each block (standard large-batch recipe).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
from torch import nn


def _conv3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride, 1, bias=False)


def _conv1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride, 0, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, width, stride=1, down: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = _conv3(cin, width, stride)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3(width, width)
        self.bn2 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, down: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = _conv1(cin, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1(width, width * 4)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = True, in_channels: int = 3):
        super().__init__()
        self.cin = 64
        self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._stage(block, 64, layers[0], 1)
        self.layer2 = self._stage(block, 128, layers[1], 2)
        self.layer3 = self._stage(block, 256, layers[2], 2)
        self.layer4 = self._stage(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _stage(self, block, width, n, stride):
        down = None
        if stride != 1 or self.cin != width * block.expansion:
            down = nn.Sequential(_conv1(self.cin, width * block.expansion, stride),
                                 nn.BatchNorm2d(width * block.expansion))
        blocks = [block(self.cin, width, stride, down)]
        self.cin = width * block.expansion
        blocks += [block(self.cin, width) for _ in range(1, n)]
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(**kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
