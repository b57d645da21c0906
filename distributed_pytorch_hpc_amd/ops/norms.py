"""RMSNorm / LayerNorm with CDNA4 kernels (csrc/rmsnorm.hip, csrc/layernorm.hip).

Reference semantics: ``RMSNorm`` of fsdp_tp/llama2_model.py:115-142 (``x.float()`` statistics,
``type_as(x)``, then ``* weight``) and ``nn.LayerNorm``.  The fused ``add_rmsnorm`` returns both the
residual sum ``h = x + r`` and ``norm(h)`` from one kernel (one fewer pass over the residual stream).
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib


# ----------------------------------------------------------------------------------------- references
def rmsnorm_reference(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).type_as(x)
    return y * w


def layernorm_reference(x, w, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


# ----------------------------------------------------------------------------------------- RMSNorm
class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, rstd, _ = _lib.ops().rmsnorm_fwd(x2, w.contiguous(), eps, None)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dx, dw = _lib.ops().rmsnorm_bwd(dy.reshape(x2.shape).contiguous(), x2, w.contiguous(), rstd)
        return dx.view(ctx.shape), dw, None


class _AddRMSNormFn(torch.autograd.Function):
    """h = x + r ; y = rmsnorm(h) * w.  Returns (h, y)."""

    @staticmethod
    def forward(ctx, x, r, w, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = r.reshape(-1, shape[-1]).contiguous()
        y, rstd, h = _lib.ops().rmsnorm_fwd(x2, w.contiguous(), eps, r2)
        ctx.save_for_backward(h, w, rstd)
        ctx.shape = shape
        return h.view(shape), y.view(shape)

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        dres = dh.reshape(h.shape).contiguous() if dh is not None else None
        dx, dw = _lib.ops().rmsnorm_bwd(dy.reshape(h.shape).contiguous(), h, w.contiguous(), rstd, dres)
        dx = dx.view(ctx.shape)
        return dx, dx, dw, None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if _lib.use_native(x) and x.shape[-1] % 8 == 0:
        return _RMSNormFn.apply(x, w, eps)
    return rmsnorm_reference(x, w, eps)


def add_rms_norm(x: torch.Tensor, r: torch.Tensor, w: torch.Tensor, eps: float = 1e-5):
    """Fused residual add + RMSNorm: returns (x + r, rmsnorm(x + r) * w)."""
    if _lib.use_native(x) and x.shape[-1] % 8 == 0:
        return _AddRMSNormFn.apply(x, r, w, eps)
    h = x + r
    return h, rmsnorm_reference(h, w, eps)


class RMSNorm(nn.Module):
    """Drop-in for the reference ``RMSNorm(dim, eps)`` (weight initialised to ones)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x, residual: "torch.Tensor | None" = None):
        """``norm(x)``; with ``residual`` the fused pre-norm step ``(x + residual, norm(x + residual))``.
        Models call the module (not the functional op on ``.weight``) so parameter-gathering forward
        pre-hooks (sharded data parallel, FSDP units) see every use of the weight."""
        if residual is None:
            return rms_norm(x, self.weight, self.eps)
        return add_rms_norm(x, residual, self.weight, self.eps)

    def reset_parameters(self):
        nn.init.ones_(self.weight)


# ----------------------------------------------------------------------------------------- LayerNorm
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = _lib.ops().layernorm_fwd(x2, w.contiguous(), b.contiguous(), eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _lib.ops().layernorm_bwd(dy.reshape(x2.shape).contiguous(), x2, w.contiguous(), mean, rstd)
        return dx.view(ctx.shape), dw, db, None


def layer_norm(x, w, b, eps=1e-5):
    d = x.shape[-1]
    if _lib.use_native(x) and d % 8 == 0 and d <= 8192 and w is not None and b is not None:
        return _LayerNormFn.apply(x, w, b, eps)
    return layernorm_reference(x, w, b, eps)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm with the CDNA4 kernel on GPU tensors."""

    def forward(self, x):
        if self.elementwise_affine and self.bias is not None:
            return layer_norm(x, self.weight, self.bias, self.eps)
        return super().forward(x)
