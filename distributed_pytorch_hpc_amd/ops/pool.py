"""Stride-2 max pooling for channels-last activations (csrc/pool.hip): 3x3 / padding 1 and 2x2 / padding 0.

``MaxPool2d`` is a drop-in ``nn.MaxPool2d`` (no parameters, same module tree): for the ResNet stem's
``MaxPool2d(3, 2, 1)`` (reference scripts/main.py:249 builds torchvision resnet50, whose stem is conv 7x7/2 -> BN ->
ReLU -> max-pool 3x3/2/1) and SimpleUNet's ``MaxPool2d(2)`` (multinode_ddp_unet.py:171-214) on a channels-last GPU
tensor with C % 8 == 0 it runs the HIP kernels: the forward keeps the window position of each max as one byte, the
backward gathers the gradient per input pixel (deterministic, no atomics, no zero-fill).  Any other configuration,
or CPU tensors, take ``F.max_pool2d``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib


def maxpool3s2_native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32) and _lib.use_native(x)
            and x.shape[1] % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and x.data_ptr() % 16 == 0)


class SkipGradSlot:
    """Hand-off of a SimpleUNet skip connection's gradient into the max-pooling backward of the same encoder output.

    An encoder output e feeds the pooling and, as the skip, the decoder's up-sample + concat (ops/upsample.py);
    autograd would sum the two gradients of e with a separate add kernel, after the concat's backward copied the skip's
    slice out of d(concat).  With a slot, the pooling (on the kernel path) marks itself the ``pool`` in its forward,
    the concat ``arms`` the slot in its own forward, and its backward -- which runs first -- leaves d(concat) in ``t``
    (skip channels from ``off``) instead of returning the slice; the pooling's gather adds it before its store
    (bitwise the bf16 sum autograd would form), so e receives one gradient and the slice is never copied."""

    __slots__ = ("pool", "armed", "t", "off")

    def __init__(self):
        self.pool = self.armed = False
        self.t = None
        self.off = 0


class _MaxPoolS2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, bn_slot=None, skip_slot=None):
        y, tap = _lib.ops().maxpool_s2_fwd(x, k)
        ctx.save_for_backward(tap)
        ctx.hw, ctx.k, ctx.bn_slot = (x.shape[2], x.shape[3]), k, bn_slot
        ctx.skip_slot = skip_slot
        if skip_slot is not None:
            skip_slot.pool = True
        return y

    @staticmethod
    def backward(ctx, dy):
        (tap,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        add, off = None, 0
        s = ctx.skip_slot
        if s is not None and s.armed:
            if s.t is None:
                raise RuntimeError("MaxPool2d: skip gradient slot armed but empty (backward order)")
            add, off = s.t, s.off
            s.t, s.armed = None, False
        bn = ctx.bn_slot   # x is a BatchNorm + ReLU output: that BatchNorm's reduction runs in this gather
        n, c = dy.shape[0], dy.shape[1]
        if (bn is not None and bn.ss is not None and dy.dtype == torch.bfloat16 and 256 % (c // 8) == 0
                and bn.usable(n * ctx.hw[0] * ctx.hw[1], c)):
            dx, bn.part = _lib.ops().maxpool_s2_bwd_bnred(dy, tap, ctx.hw[0], ctx.hw[1], ctx.k, bn.x, bn.mean,
                                                          bn.invstd, bn.ss, add, off)
            bn.mark(dx)
            return dx, None, None, None
        return _lib.ops().maxpool_s2_bwd(dy, tap, ctx.hw[0], ctx.hw[1], ctx.k, add, off), None, None, None


def max_pool3s2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, 1)`` with the HIP kernels when eligible."""
    if maxpool3s2_native_ok(x):
        return _MaxPoolS2Fn.apply(x, 3)
    return F.max_pool2d(x, 3, 2, 1)


def max_pool2s2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 2)`` with the HIP kernels when eligible."""
    if maxpool3s2_native_ok(x) and x.shape[2] >= 2 and x.shape[3] >= 2:
        return _MaxPoolS2Fn.apply(x, 2)
    return F.max_pool2d(x, 2)


class MaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` whose 3x3 / stride 2 / padding 1 and 2x2 / stride 2 cases run the channels-last HIP
    kernels."""

    def forward(self, x, bn_slot=None, skip_slot=None):
        """``bn_slot`` (ops.conv.BnGradSlot): x is a training-mode BatchNorm + ReLU output (the ResNet stem, a
        SimpleUNet encoder block); the BatchNorm's backward reduction then runs in this pooling's gradient gather.
        ``skip_slot`` (SkipGradSlot): x is also a SimpleUNet skip connection; its gradient is added in the gather."""
        k = {(3, 1): 3, (2, 0): 2}.get((_one(self.kernel_size), _one(self.padding)))
        fast = (k is not None and _one(self.stride) == 2 and _one(self.dilation) == 1 and not self.ceil_mode
                and not self.return_indices)
        if fast and maxpool3s2_native_ok(x) and x.shape[2] >= k - 1 and x.shape[3] >= k - 1:
            return _MaxPoolS2Fn.apply(x, k, bn_slot, skip_slot)
        return super().forward(x)


def _one(v):
    """A square pooling parameter as an int (None when the two dimensions differ)."""
    if isinstance(v, (tuple, list)):
        return v[0] if len(set(v)) == 1 else None
    return v
