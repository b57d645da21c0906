"""ResNet-18/34/50/101/152, defined natively (torchvision is not installed in this environment).

Capability parity with the torchvision models the reference trains (scripts/main.py:186-191,249 -- resnet18/50/101/152
with pretrained=False; scripts/02_fully_sharded_fsdp/resnet_fsdp_training.py:186-191 -- ResNet-18 with the CIFAR stem:
3x3 stride-1 conv1 and no max-pool).  The module tree and parameter names match torchvision
(conv1, bn1, layer1..4[i].{conv1..3, bn1..3, downsample.{0,1}}, fc), so torchvision state dicts load directly and
the parameter counts agree (ResNet-50: 25,557,032).

MI355X-first choices: ``channels_last=True`` keeps activations NHWC (MIOpen's implicit-GEMM layout) end to end,
every BN -> (+identity) -> ReLU runs as one fused channels-last HIP op (ops.batchnorm.BatchNormAct2d: one stats
pass + one apply pass forward, the residual's gradient produced by the BN backward), and ``zero_init_residual`` is
available (as torchvision).  ``BatchNormAct2d`` subclasses ``nn.BatchNorm2d``, so the state-dict keys are unchanged.
"""
from __future__ import annotations

from typing import Type, Union

import torch
from torch import nn

from ..ops.batchnorm import BatchNormAct2d
from ..ops.batchnorm import bn_dual_act, bn_relu_conv1x1, bn_relu_conv1x1_ok
from ..ops.conv import (BnGradSlot, Conv1x1, Conv3x3, GradSlot, StatsSlot, StemConv2d, StridedConv2d, grad_tap,
                        strided_native_ok)
from ..ops.pool import MaxPool2d


def conv3x3(cin, cout, stride=1):
    # channels-last implicit-GEMM kernel paths (ops/conv.py): stride 1 Conv3x3, strided the gathered-row kernels
    return Conv3x3(cin, cout) if stride == 1 else StridedConv2d(cin, cout, 3, stride, 1, bias=False)


def conv1x1(cin, cout, stride=1):
    # nn.Conv2d-compatible modules that run channels-last bf16 on the CDNA4 GEMM kernels (ops/conv.py); the strided
    # 1x1 (the downsample of layers 2-4) gathers every s-th pixel in its operand load
    return Conv1x1(cin, cout) if stride == 1 else StridedConv2d(cin, cout, 1, stride, 0, bias=False)


class BnHandoff:
    """Hands a block's last BatchNorm slot (ops.conv.BnGradSlot) to the next block's conv1, which consumes that output.

    A tensor attribute would not survive module hooks (full backward hooks hand the next block an alias of the
    output), so the producing block leaves the slot here with the output's storage key, and the consuming block takes
    it only when its input has that key (same storage, shape and strides).  Plain object (not a Module): no state."""

    __slots__ = ("slot", "key")

    def __init__(self):
        self.slot = self.key = None

    @staticmethod
    def _key(t: torch.Tensor):
        return (t.data_ptr(), tuple(t.shape), tuple(t.stride()))

    def put(self, y: torch.Tensor, slot):
        self.slot, self.key = slot, (self._key(y) if slot is not None else None)

    def take(self, x: torch.Tensor):
        slot, key = self.slot, self.key
        self.slot = self.key = None
        return slot if slot is not None and key == self._key(x) else None


def link_bn_handoff(blocks) -> None:
    """Chain consecutive bottleneck blocks (in forward order) through one BnHandoff (ResNet does this for its own)."""
    h = BnHandoff()
    for b in blocks:
        if isinstance(b, Bottleneck):
            b._dph_handoff = h


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = BatchNormAct2d(planes)                  # relu(bn1(.))
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = BatchNormAct2d(planes)                  # relu(bn2(.) + identity)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        # bn1's backward reduction runs in conv2's input-gradient epilogue (its only consumer; ops.conv.BnGradSlot)
        r1 = BnGradSlot() if isinstance(self.conv2, Conv3x3) and self.bn1.training else None
        out = self.bn1(self.conv1(x), bn_slot=r1)
        return self.bn2(self.conv2(out, bn_slot=r1), idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = BatchNormAct2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = BatchNormAct2d(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = BatchNormAct2d(planes * 4)              # relu(bn3(.) + identity)
        self.downsample = downsample

    def forward(self, x):
        # conv1's input-gradient kernel also adds x's other gradient (ops.conv.GradSlot): bn3's residual gradient in
        # identity blocks, the downsample convolution's input gradient in downsample blocks
        slot = None
        if isinstance(self.conv1, Conv1x1) and x.requires_grad and torch.is_grad_enabled():
            slot = GradSlot()
        # training-mode BN after a 1x1 convolution takes its statistics from the convolution's epilogue
        s1 = StatsSlot() if self.bn1.training and isinstance(self.conv1, Conv1x1) else None
        s3 = StatsSlot() if self.bn3.training and isinstance(self.conv3, Conv1x1) else None
        # BatchNorm backward reductions in the consuming convolution's input-gradient epilogue (ops.conv.BnGradSlot):
        # bn1 -> conv2 (stride-1 3x3), bn2 -> conv3, and the previous block's bn3 -> this conv1 when the GradSlot
        # carries x's other gradient (identity or downsample) into the same epilogue
        train = self.bn1.training
        r1 = BnGradSlot() if train and isinstance(self.conv2, Conv3x3) else None
        r2 = BnGradSlot() if train and isinstance(self.conv3, Conv1x1) else None
        r3 = BnGradSlot(sole=False) if self.bn3.training else None
        hand = getattr(self, "_dph_handoff", None)
        rin = hand.take(x) if hand is not None and slot is not None else None
        out = self.bn1(self.conv1(x, grad_slot=slot, stats_slot=s1, bn_slot=rin), stats_slot=s1, bn_slot=r1)
        z = dbn = None
        if self.downsample is None:
            idt, res_slot = x, slot
        else:
            # built after conv1 / bn1, so autograd runs the downsample branch's backward (ending in the tap) before
            # conv1's: the tap parks the branch's gradient of x for conv1's dgrad epilogue (no separate add over x)
            ds = self.downsample[0]
            if (len(self.downsample) == 2 and isinstance(self.downsample[1], BatchNormAct2d)
                    and isinstance(ds, (Conv1x1, StridedConv2d))):
                # projection shortcut: the downsample BatchNorm takes its statistics from the convolution's epilogue
                # and is applied inside bn3's apply pass (ops.batchnorm.bn_dual_act) -- its output never written
                dbn = self.downsample[1]
                sds = StatsSlot() if dbn.training else None
            if (slot is not None and slot.consumer and isinstance(ds, StridedConv2d) and ds.kernel_size == (1, 1)
                    and ds.stride == (2, 2) and strided_native_ok(x, ds)):
                # strided 1x1 downsample: its sub-image input gradient goes to conv1's epilogue (added at the even
                # pixels), so no zero-filled full-size gradient of x is ever written
                slot.armed = True
                z = ds(x, stats_slot=sds if dbn is not None else None, grad_slot=slot)
            else:
                tapped = grad_tap(x, slot) if slot is not None and slot.consumer else x
                z = ds(tapped, stats_slot=sds) if dbn is not None else ds(tapped)
            if dbn is None:
                idt, z = self.downsample[1:](z), None
            res_slot = None
        s2 = StatsSlot() if isinstance(self.conv2, (Conv3x3, StridedConv2d)) and self.bn2.training else None
        if isinstance(self.conv2, Conv3x3):
            out = self.conv2(out, stats_slot=s2, bn_slot=r1)
        else:
            out = self.conv2(out, stats_slot=s2) if s2 is not None else self.conv2(out)
        if bn_relu_conv1x1_ok(self.bn2, self.conv3, out):
            # bn2's apply + ReLU folded into conv3's operand loads (forward and weight gradient): the normalised
            # activation is never written (ops.batchnorm._BNReLUConv1x1Fn)
            out = bn_relu_conv1x1(self.bn2, self.conv3, out, s2, s3)
        else:
            out = self.conv3(self.bn2(out, stats_slot=s2, bn_slot=r2), stats_slot=s3, bn_slot=r2)
        if z is not None:
            y = bn_dual_act(self.bn3, dbn, out, z, s3, sds, r3)
        else:
            y = self.bn3(out, idt, residual_grad_slot=res_slot, stats_slot=s3, bn_slot=r3)
        if hand is not None:
            hand.put(y, r3)   # for the next block's conv1
        return y


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: list[int], num_classes: int = 1000,
                 cifar_stem: bool = False, zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        if cifar_stem:
            self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
            self.maxpool = nn.Identity()
        else:
            self.conv1 = StemConv2d(3, 64, 7, 2, 3, bias=False)   # 4-channel NHWC padding on the GPU (ops/conv.py)
            self.maxpool = MaxPool2d(3, 2, 1)   # channels-last HIP kernels (ops/pool.py)
        self.bn1 = BatchNormAct2d(64)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        link_bn_handoff([b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer])
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
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

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 BatchNormAct2d(planes * block.expansion, act=False))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        if isinstance(self.conv1, StemConv2d) and self.bn1.training:
            # the stem's GEMM epilogue hands bn1 its batch statistics (no statistics pass over the 112^2 activation)
            s = StatsSlot()
            r0 = BnGradSlot() if isinstance(self.maxpool, MaxPool2d) else None   # reduction in the pool's gather
            y = self.bn1(self.conv1(x, stats_slot=s), stats_slot=s, bn_slot=r0)
            x = self.maxpool(y, bn_slot=r0) if r0 is not None else self.maxpool(y)
        else:
            x = self.maxpool(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


_CFG = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
    "resnet152": (Bottleneck, [3, 8, 36, 3]),
}


def resnet(arch: str = "resnet50", num_classes: int = 1000, cifar_stem: bool = False, channels_last: bool = False,
           **kw) -> ResNet:
    block, layers = _CFG[arch]
    m = ResNet(block, layers, num_classes=num_classes, cifar_stem=cifar_stem, **kw)
    return m.to(memory_format=torch.channels_last) if channels_last else m


def resnet18(**kw):
    return resnet("resnet18", **kw)


def resnet50(**kw):
    return resnet("resnet50", **kw)


def resnet101(**kw):
    return resnet("resnet101", **kw)


def resnet152(**kw):
    return resnet("resnet152", **kw)
