"""Rotary position embedding, interleaved-pair convention of fsdp_tp/llama2_model.py:30-100.

The reference builds a complex64 ``freqs_cis`` table and multiplies ``view_as_complex`` pairs
(x[2i], x[2i+1]).  Here the host precomputes fp32 cos/sin tables once and the HIP kernel
(csrc/elementwise.hip rope_k) rotates in place on strided [B, S, H, hd] views, so q and k can be
rotated directly inside the fused QKV GEMM output without a layout copy.
"""
from __future__ import annotations

import torch

from . import _lib


def precompute_rope_tables(head_dim: int, max_pos: int, theta: float = 10000.0, device=None):
    """fp32 cos/sin tables of shape [max_pos, head_dim // 2] (angles computed in fp64 on the host)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64)[: head_dim // 2] / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos_offset: int = 0, inverse=False):
    """Out-of-place reference on [B, S, H, hd] (fp32 math, cast back)."""
    s = x.shape[1]
    c = cos[pos_offset: pos_offset + s].view(1, s, 1, -1)
    sn = sin[pos_offset: pos_offset + s].view(1, s, 1, -1)
    if inverse:
        sn = -sn
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    a, b = xf[..., 0], xf[..., 1]
    out = torch.stack((a * c - b * sn, a * sn + b * c), dim=-1).flatten(-2)
    return out.type_as(x)


def rope_(x: torch.Tensor, cos, sin, pos_offset: int = 0, inverse: bool = False) -> torch.Tensor:
    """In-place rotation of a [B, S, H, hd] (possibly strided) view; no autograd."""
    if _lib.use_native(x) and x.shape[-1] % 8 == 0:
        _lib.ops().rope_(x, cos, sin, pos_offset, inverse)
        return x
    x.copy_(rope_reference(x, cos, sin, pos_offset, inverse))
    return x


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos_offset):
        ctx.cs = (cos, sin, pos_offset)
        return rope_(x.clone(), cos, sin, pos_offset, False)

    @staticmethod
    def backward(ctx, g):
        cos, sin, off = ctx.cs
        return rope_(g.clone(), cos, sin, off, True), None, None, None


def apply_rope(x: torch.Tensor, cos, sin, pos_offset: int = 0) -> torch.Tensor:
    """Autograd-aware out-of-place RoPE on [B, S, H, hd]."""
    return _RopeFn.apply(x, cos, sin, pos_offset)
