"""ResNet-50 (v1.5: stride on the 3x3 conv) -- the BASELINE.json headline model.

torchvision is not in the image, so the architecture is defined here (He et al. 2016,
torchvision layer naming so state dicts line up).  Random init only (no checkpoints).

MI355X notes: the model is run in channels_last bf16 (MIOpen NHWC convolutions on the
MFMA cores); all parameters -- conv, BN and FC -- are bf16 replicas whose fp32 masters
live on the parameter-server shards (parallel/colocated.py).  BN running statistics are
fp32 buffers kept per worker (they are not trained parameters, so they are not pushed;
the reference has no BN at all).
"""
from __future__ import annotations


import torch
import torch.nn as nn

from .. import knobs
from ..ops.bn import BatchNormAct2d
from ..ops.conv import Conv1x1, StemConv, stem_bn_relu_maxpool
from ..ops.convgemm import (deferred_bn_counters, flush_deferred, fused_block_ok, fused_bottleneck,
                             prepare_backward_weights, resp_consumer_ok)
from ..ops.pool import MaxPool2d, global_avg_pool


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None,
                 fused_bn: bool = True):
        super().__init__()
        width = planes
        self.fused_bn = fused_bn
        BN = BatchNormAct2d if fused_bn else nn.BatchNorm2d
        C1 = Conv1x1 if fused_bn else (lambda i, o: nn.Conv2d(i, o, 1, bias=False))
        self.conv1 = C1(inplanes, width)
        self.bn1 = BN(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BN(width)
        self.conv3 = C1(width, planes * 4)
        self.bn3 = BN(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        # whole-block fused path (implicit-GEMM 1x1 convs with the BN passes folded in,
        # ops/convgemm.py) for GPU bf16 training; the module path below otherwise
        self.fuse_block = fused_bn

    def forward(self, x):
        if self.fuse_block and fused_block_ok(self, x):
            return fused_bottleneck(self, x)
        flush_deferred()  # a deferred fused-block output (never on the fused ResNet path)
        identity = x if self.downsample is None else self.downsample(x)
        if self.fused_bn:
            # BN + ReLU fused; bn3 fuses the residual add and the final ReLU (ops/bn.py)
            out = self.bn1(self.conv1(x))
            out = self.bn2(self.conv2(out))
            return self.bn3(self.conv3(out), identity)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, zero_init_residual: bool = True,
                 fused_bn: bool = True):
        super().__init__()
        self.inplanes = 64
        self.fused_bn = fused_bn
        self.conv1 = StemConv(3) if fused_bn else nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(64) if fused_bn else nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = (MaxPool2d if fused_bn else nn.MaxPool2d)(3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
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

    def _blocks(self):
        return [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            bn = BatchNormAct2d(planes * 4, act="none") if self.fused_bn else nn.BatchNorm2d(planes * 4)
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False), bn)
        layers = [Bottleneck(self.inplanes, planes, stride, downsample, self.fused_bn)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes, fused_bn=self.fused_bn))
        return nn.Sequential(*layers)

    def forward(self, x):
        if self.fused_bn:  # stem BN + ReLU fused into the pool: the BN output never hits HBM
            x = stem_bn_relu_maxpool(x, self.conv1, self.bn1)
        else:
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        with deferred_bn_counters():
            if self.fused_bn and self.training and x.is_cuda:
                blks = self._blocks()
                prepare_backward_weights(blks)  # all data-grad weight layouts, one kernel
                # a block followed by a fused block leaves its output to that block's conv1 prologue
                # where that pays (ops/convgemm.py resp_consumer_ok)
                on = knobs.enabled("block_out")
                h, w = x.shape[2], x.shape[3]
                for a, b in zip(blks, blks[1:] + [None]):
                    s = a.conv2.stride[0]
                    h, w = (h - 1) // s + 1, (w - 1) // s + 1  # a's output map = b's input map
                    a._defer_out = (on and b is not None and b.fuse_block
                                    and resp_consumer_ok(b, x.shape[0] * h * w))
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.fused_bn:
            x = global_avg_pool(x)  # NHWC gradient straight into the last block's backward
        else:
            x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet50(num_classes: int = 1000, fused_bn: bool = True) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes, fused_bn=fused_bn)


def resnet_tiny(num_classes: int = 10, fused_bn: bool = True) -> ResNet:
    """One bottleneck per stage: same code path as ResNet-50 for quick tests."""
    return ResNet((1, 1, 1, 1), num_classes, fused_bn=fused_bn)


def prepare_for_mi355x(model: nn.Module, dtype=torch.bfloat16, bn_fp32: bool = True) -> nn.Module:
    """channels_last + bf16 parameters.

    bn_fp32=True keeps BatchNorm affine params and running stats in fp32 (the mixed
    bf16-activation / fp32-BN-param path that MIOpen and the native kernels both support);
    bn_fp32=False casts the whole module, BN included, to ``dtype``.
    """
    model = model.to(memory_format=torch.channels_last)
    for mod in model.modules():
        is_bn = isinstance(mod, nn.modules.batchnorm._BatchNorm)
        if is_bn and bn_fp32:
            continue
        for _, p in list(mod.named_parameters(recurse=False)):
            p.data = p.data.to(dtype)
        for name, b in list(mod.named_buffers(recurse=False)):
            if b.is_floating_point():
                setattr(mod, name, b.to(dtype))
    return model
