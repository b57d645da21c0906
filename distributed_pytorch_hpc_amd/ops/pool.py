"""3x3 / stride 2 / padding 1 max pooling for channels-last activations (csrc/pool.hip).

``MaxPool2d`` is a drop-in ``nn.MaxPool2d`` (no parameters, same module tree): for the ResNet stem's
``MaxPool2d(3, 2, 1)`` (reference scripts/main.py:249 builds torchvision resnet50, whose stem is conv 7x7/2 -> BN ->
ReLU -> max-pool 3x3/2/1) on a channels-last GPU tensor with C % 8 == 0 it runs the HIP kernels: the forward keeps
the window position of each max as one byte, the backward gathers the gradient per input pixel (deterministic, no
atomics, no zero-fill).  Any other configuration, or CPU tensors, take ``F.max_pool2d``.
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


class _MaxPool3s2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, tap = _lib.ops().maxpool3s2_fwd(x)
        ctx.save_for_backward(tap)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        (tap,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        return _lib.ops().maxpool3s2_bwd(dy, tap, ctx.hw[0], ctx.hw[1])


def max_pool3s2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, 1)`` with the HIP kernels when eligible."""
    if maxpool3s2_native_ok(x):
        return _MaxPool3s2Fn.apply(x)
    return F.max_pool2d(x, 3, 2, 1)


class MaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` whose 3x3 / stride 2 / padding 1 case runs the channels-last HIP kernels."""

    def forward(self, x):
        fast = (self.kernel_size in (3, (3, 3)) and self.stride in (2, (2, 2)) and self.padding in (1, (1, 1))
                and self.dilation in (1, (1, 1)) and not self.ceil_mode and not self.return_indices)
        if fast and maxpool3s2_native_ok(x):
            return _MaxPool3s2Fn.apply(x)
        return super().forward(x)
