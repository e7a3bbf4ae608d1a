"""ResNet family (He et al. 2015, v1.5: stride on the 3x3 conv), defined in-repo
(torchvision is not available).  ResNet-50 = 25,557,032 parameters in 161 tensors.

``gemm_1x1=True`` runs the stride-1 1x1 convs as hipBLASLt GEMMs and the
3x3 convs and the stride-2 1x1 projections on the MFMA implicit-GEMM kernels
(ops/conv.py).
``fused_bn=True`` replaces each BatchNorm(+ReLU)(+residual add) with the fused
gfx950 op ``BatchNorm2dReLU`` (one stats pass + one elementwise pass forward,
one reduction + one elementwise pass backward, ReLU and the residual add folded
in).  With ``channels_last`` activations the NHWC kernels run, which is the
layout MIOpen's bf16 convolutions prefer on MI355X.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from ..ops.batch_norm import BatchNorm2dReLU
from ..ops.batch_norm import bn_add_bn_relu
from ..ops.conv import Conv2d1x1, Conv2d3x3, StemConv2d, conv1x1_pair_s2
from ..ops.pool import (GlobalAvgPool2dNHWC, MaxPool2dNHWC, bn_relu_maxpool,
                        bn_relu_maxpool_fusable)


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1, mfma=False):
    if mfma and stride in (1, 2) and groups == 1 and dilation == 1:
        return Conv2d3x3(in_planes, out_planes, stride)
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                     groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1, gemm=False):
    if gemm:
        return Conv2d1x1(in_planes, out_planes, stride=stride)
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class _BNAct(nn.Module):
    """BN (+ residual) (+ ReLU): plain torch modules or the fused op."""

    def __init__(self, planes, relu, fused, zero_init=False):
        super().__init__()
        self.fused = fused
        self.relu_after = relu
        if fused:
            self.bn = BatchNorm2dReLU(planes, fuse_relu=relu)
        else:
            self.bn = nn.BatchNorm2d(planes)
        if zero_init:
            nn.init.zeros_(self.bn.weight)

    def forward(self, x, z=None):
        if self.fused:
            return self.bn(x, z)
        y = self.bn(x)
        if z is not None:
            y = y + z
        return torch.relu(y) if self.relu_after else y


def _link_stats(conv, bnact):
    """Let ``conv`` write the BatchNorm statistics of its output for ``bnact.bn`` in its
    epilogue (ops/conv.py; resolved at forward time, so convert_syncbn_model's
    replacement BN is the one that receives them)."""
    if bnact.fused:
        conv._amd_stats_bn = weakref.ref(bnact)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, fused_bn=False,
                 zero_init_residual=False, gemm_1x1=False):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride, mfma=gemm_1x1)
        self.bn1 = _BNAct(planes, True, fused_bn)
        self.conv2 = conv3x3(planes, planes, mfma=gemm_1x1)
        self.bn2 = _BNAct(planes, True, fused_bn, zero_init_residual)
        self.downsample = downsample
        _link_stats(self.conv1, self.bn1)
        _link_stats(self.conv2, self.bn2)

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.bn1(self.conv1(x))
        return self.bn2(self.conv2(out), identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, fused_bn=False,
                 zero_init_residual=False, gemm_1x1=False):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width, gemm=gemm_1x1)
        self.bn1 = _BNAct(width, True, fused_bn)
        self.conv2 = conv3x3(width, width, stride, mfma=gemm_1x1)
        self.bn2 = _BNAct(width, True, fused_bn)
        self.conv3 = conv1x1(width, planes * self.expansion, gemm=gemm_1x1)
        self.bn3 = _BNAct(planes * self.expansion, True, fused_bn, zero_init_residual)
        self.downsample = downsample
        _link_stats(self.conv1, self.bn1)
        _link_stats(self.conv2, self.bn2)
        _link_stats(self.conv3, self.bn3)

    def forward(self, x):
        # downsample block with fused BNs: the projection's BN is applied inside bn3's pass
        # (ops/batch_norm.py bn_add_bn_relu), its output never materialised
        fuse_ds = self.downsample is not None and self.bn3.fused and self.downsample.bn.fused
        proj = identity = None
        if (isinstance(self.conv1, Conv2d1x1) and self.downsample is not None
                and self.downsample.conv.stride == (2, 2)):
            # conv1 and the stride-2 downsample projection read the same input: one
            # Function keeps the projection's input gradient compact (strided pixels
            # only) and conv1's dgrad adds it on the even pixels (ops/conv.py)
            out, proj = conv1x1_pair_s2(self.conv1, self.downsample.conv, x)
        elif isinstance(self.conv1, Conv2d1x1):
            # the block input feeds conv1 and the residual branch (identity or the
            # downsample conv): the two input gradients are summed inside conv1's
            # dgrad GEMM (C += dY @ W into the branch's gradient), not by a separate
            # add kernel over the block input
            out, skip = self.conv1.forward_with_skip(x)
            if self.downsample is None:
                identity = skip
            else:
                proj = self.downsample.conv(skip)
        else:
            if self.downsample is None:
                identity = x
            else:
                proj = self.downsample.conv(x)
            out = self.conv1(x)
        if proj is not None and not fuse_ds:
            identity = self.downsample.bn(proj)
        out = self.bn1(out)
        out = self.bn2(self.conv2(out))
        if proj is not None and fuse_ds:
            return bn_add_bn_relu(self.bn3.bn, self.conv3(out), self.downsample.bn.bn, proj)
        return self.bn3(self.conv3(out), identity)


class _Downsample(nn.Module):
    def __init__(self, inplanes, outplanes, stride, fused_bn, gemm_1x1=False):
        super().__init__()
        self.conv = conv1x1(inplanes, outplanes, stride, gemm=gemm_1x1)
        self.bn = _BNAct(outplanes, False, fused_bn)
        _link_stats(self.conv, self.bn)

    def forward(self, x):
        return self.bn(self.conv(x))


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, fused_bn=False, zero_init_residual=False,
                 gemm_1x1=False):
        super().__init__()
        self.fused_bn = fused_bn
        self.gemm_1x1 = gemm_1x1
        self.inplanes = 64
        if gemm_1x1 and self.inplanes == 64:
            self.conv1 = StemConv2d(3, self.inplanes)  # MFMA stem kernels (ops/conv.py)
        else:
            self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3,
                                   bias=False)
        self.bn1 = _BNAct(self.inplanes, True, fused_bn)
        if isinstance(self.conv1, StemConv2d):
            _link_stats(self.conv1, self.bn1)  # stem BN statistics from the stem epilogue
        pool = MaxPool2dNHWC if fused_bn else nn.MaxPool2d
        self.maxpool = pool(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0], 1, zero_init_residual)
        self.layer2 = self._make_layer(block, 128, layers[1], 2, zero_init_residual)
        self.layer3 = self._make_layer(block, 256, layers[2], 2, zero_init_residual)
        self.layer4 = self._make_layer(block, 512, layers[3], 2, zero_init_residual)
        self.avgpool = GlobalAvgPool2dNHWC() if fused_bn else nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make_layer(self, block, planes, blocks, stride, zero_init_residual):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = _Downsample(self.inplanes, planes * block.expansion, stride,
                                     self.fused_bn, self.gemm_1x1)
        layers = [block(self.inplanes, planes, stride, downsample, self.fused_bn,
                        zero_init_residual, self.gemm_1x1)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, fused_bn=self.fused_bn,
                                zero_init_residual=zero_init_residual, gemm_1x1=self.gemm_1x1))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.conv1(x)
        if (self.fused_bn and isinstance(self.maxpool, MaxPool2dNHWC)
                and bn_relu_maxpool_fusable(x, self.bn1.bn, self.maxpool)):
            # stem BN + ReLU applied inside the max-pool's loads (never materialised)
            x = bn_relu_maxpool(x, self.bn1.bn, self.maxpool)
        else:
            x = self.maxpool(self.bn1(x))
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        x = self.avgpool(x)
        x = torch.flatten(x, 1)
        return self.fc(x)


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
