"""SimpleUNet for ERA5-style gridded data (capability parity with
scripts/01_data_parallel_ddp/multinode_ddp_unet.py:171-214; 7,742,849 parameters at 65 -> 65 channels).

Same modules and names (enc1..3, bottleneck, up1..3, dec1..3, out, pool).  Convolutions run through MIOpen in
channels-last (NHWC) layout when the model is moved to the GPU with ``to_channels_last`` -- the MI355X-native
layout for implicit-GEMM convolutions; the odd 181-latitude grid is handled like the reference (bilinear
resize of each up-sampled map to its skip connection size), with transposed convolution + resize + concat run as one
GEMM and one copy kernel per decoder level (ops/upsample.py, csrc/upsample.hip).  ``halo`` (domain parallelism, parallel/domain.py)
swaps the 3x3 convolutions for halo-exchanging ones when the latitude axis is sharded across ranks.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from ..ops.batchnorm import BatchNormAct2d
from ..ops.conv import BiasConv2d, BiasConvTranspose2d, BnGradSlot, StatsSlot
from ..ops.pool import MaxPool2d, SkipGradSlot
from ..ops.upsample import up_concat


class ConvBlock(nn.Sequential):
    """conv -> BN -> ReLU twice, as the reference's ``conv_block``; BN + ReLU run as one fused channels-last op
    (BatchNormAct2d, a BatchNorm2d subclass: same state-dict keys; the ReLU slots stay as Identity so the indices are
    unchanged), and a training-mode BN takes its batch statistics from the 3x3 convolution's epilogue (StatsSlot)
    instead of a statistics pass over the activation."""

    def out_slot(self, y: torch.Tensor):
        """The second BatchNorm's slot (ops.conv.BnGradSlot) if ``y`` is this block's last output -- for a consumer
        that receives the output's whole gradient: the up-path GEMM after the bottleneck and the decoder blocks, the
        output convolution, and an encoder block's max pooling when the skip connection's gradient is added in its
        gather (ops.pool.SkipGradSlot)."""
        slot, key = getattr(self, "_dph_out", (None, None))
        self._dph_out = (None, None)
        if os.environ.get("DPH_UNET_OUT_FOLD", "1") == "0":   # A/B: those BatchNorms run their own reduction pass
            return None
        return slot if slot is not None and key == (y.data_ptr(), tuple(y.shape), tuple(y.stride())) else None

    def forward(self, x):
        # the first BatchNorm's output is consumed only by the second convolution: its backward reduction runs in that
        # convolution's input-gradient epilogue (ops.conv.BnGradSlot); the second's is offered to the block's
        # consumer (out_slot)
        red = None
        self._dph_out = (None, None)
        for i, (conv, bn) in enumerate(((self[0], self[1]), (self[3], self[4]))):
            if isinstance(conv, BiasConv2d) and isinstance(bn, BatchNormAct2d) and bn.training:
                slot = StatsSlot()
                nxt = BnGradSlot() if i == 1 or isinstance(self[3], BiasConv2d) else None
                x = bn(conv(x, stats_slot=slot, bn_slot=red), stats_slot=slot, bn_slot=nxt)
                red = nxt
                if i == 1 and nxt is not None:
                    self._dph_out = (nxt, (x.data_ptr(), tuple(x.shape), tuple(x.stride())))
            else:   # modules swapped in by a wrapper (e.g. the halo convolutions of parallel/domain.py)
                x = bn(conv(x))
                red = None
        return x


def conv_block(in_ch: int, out_ch: int) -> nn.Sequential:
    return ConvBlock(
        BiasConv2d(in_ch, out_ch, 3, padding=1), BatchNormAct2d(out_ch), nn.Identity(),
        BiasConv2d(out_ch, out_ch, 3, padding=1), BatchNormAct2d(out_ch), nn.Identity(),
    )


class SimpleUNet(nn.Module):
    def __init__(self, in_channels: int = 65, out_channels: int = 65, base_dim: int = 64):
        super().__init__()
        b = base_dim
        self.enc1 = conv_block(in_channels, b)
        self.enc2 = conv_block(b, 2 * b)
        self.enc3 = conv_block(2 * b, 4 * b)
        self.bottleneck = conv_block(4 * b, 8 * b)
        self.up3 = BiasConvTranspose2d(8 * b, 4 * b, 2, 2)
        self.dec3 = conv_block(8 * b, 4 * b)
        self.up2 = BiasConvTranspose2d(4 * b, 2 * b, 2, 2)
        self.dec2 = conv_block(4 * b, 2 * b)
        self.up1 = BiasConvTranspose2d(2 * b, b, 2, 2)
        self.dec1 = conv_block(2 * b, b)
        self.out = BiasConv2d(b, out_channels, kernel_size=1)
        self.pool = MaxPool2d(2)   # channels-last HIP kernels (ops/pool.py)

    def forward(self, x):
        # each encoder output feeds the pooling and the skip connection: the skip's gradient is added in the pooling's
        # gather (ops.pool.SkipGradSlot), which then holds e's whole gradient and so also runs the block's last
        # BatchNorm reduction
        fold = self.training and os.environ.get("DPH_UNET_SKIP_FOLD", "1") != "0"
        s1, s2, s3 = (SkipGradSlot(), SkipGradSlot(), SkipGradSlot()) if fold else (None, None, None)
        e1 = self.enc1(x)
        e2 = self.enc2(self._pool(e1, self.enc1, s1))
        e3 = self.enc3(self._pool(e2, self.enc2, s2))
        bt = self.bottleneck(self._pool(e3, self.enc3, s3))
        # up-sample + resize + concat: one GEMM and one copy kernel per level on the GPU (ops/upsample.py); the
        # bottleneck / decoder outputs feed only the next GEMM, which then runs their last BatchNorm's reduction
        d3 = self.dec3(up_concat(self.up3, bt, e3, bn_slot=_out_slot(self.bottleneck, bt), skip_slot=s3))
        d2 = self.dec2(up_concat(self.up2, d3, e2, bn_slot=_out_slot(self.dec3, d3), skip_slot=s2))
        d1 = self.dec1(up_concat(self.up1, d2, e1, bn_slot=_out_slot(self.dec2, d2), skip_slot=s1))
        if isinstance(self.out, BiasConv2d):
            return self.out(d1, bn_slot=_out_slot(self.dec1, d1))
        return self.out(d1)

    def _pool(self, e, block, skip_slot):
        if skip_slot is None or not isinstance(self.pool, MaxPool2d):
            return self.pool(e)
        return self.pool(e, bn_slot=_out_slot(block, e), skip_slot=skip_slot)


def _out_slot(block, y):
    return block.out_slot(y) if isinstance(block, ConvBlock) else None


def to_channels_last(model: nn.Module) -> nn.Module:
    return model.to(memory_format=torch.channels_last)
