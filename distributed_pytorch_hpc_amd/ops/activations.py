"""SwiGLU and GELU with CDNA4 kernels (csrc/elementwise.hip).

``swiglu(x2)`` consumes the output of the FUSED w1||w3 GEMM ([..., 2F], gate first), so the Llama
FeedForward (fsdp_tp/llama2_model.py:231-272, ``w2(silu(w1 x) * w3 x)``) runs as one GEMM + one
elementwise kernel + one GEMM, forward and backward.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def swiglu_reference(x2: torch.Tensor) -> torch.Tensor:
    g, u = x2.chunk(2, dim=-1)
    return F.silu(g) * u


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2):
        x2 = x2.contiguous()
        ctx.save_for_backward(x2)
        return _lib.ops().swiglu_fwd(x2)

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        return _lib.ops().swiglu_bwd(dy.contiguous(), x2)


def swiglu(x2: torch.Tensor) -> torch.Tensor:
    if _lib.use_native(x2) and x2.shape[-1] % 16 == 0:
        return _SwiGLUFn.apply(x2)
    return swiglu_reference(x2)


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, tanh_form):
        x = x.contiguous()
        ctx.save_for_backward(x)
        ctx.tanh_form = tanh_form
        return _lib.ops().gelu_fwd(x, tanh_form)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _lib.ops().gelu_bwd(dy.contiguous(), x, ctx.tanh_form), None


def gelu(x: torch.Tensor, approximate: str = "none") -> torch.Tensor:
    if _lib.use_native(x) and x.numel() % 8 == 0:
        return _GeluFn.apply(x, approximate == "tanh")
    return F.gelu(x, approximate=approximate)


class GELU(torch.nn.Module):
    def __init__(self, approximate: str = "none"):
        super().__init__()
        self.approximate = approximate

    def forward(self, x):
        return gelu(x, self.approximate)
