"""SimpleUNet up-path as one GEMM + one copy kernel: ConvTranspose2d(2, 2) -> bilinear resize -> concat (csrc/upsample.hip).

The reference decoder (scripts/01_data_parallel_ddp/multinode_ddp_unet.py:180-188, 205-213) runs, per level,
``up = ConvTranspose2d(k=2, s=2)(x)``, ``F.interpolate(up, size=skip.shape[2:], mode="bilinear")`` when the odd
181-row grid makes the sizes differ, and ``torch.cat([up, skip], dim=1)``: three passes over the up-sampled map (four
under bf16 autocast, which runs the resize in fp32 and promotes the cat).  Here:

* forward: ``Y' = X Wr`` on the tall-skinny GEMM of csrc/conv1x1.hip (channels-last X viewed as [N*H*W, Cin];
  ``Wr`` = the weight as [Cin, (i, j, Cout)]; hipBLASLt when the channel counts are not multiples of 64), then ``upcat_fwd`` writes the concatenated decoder input directly: the bilinear sample of the
  pixel-shuffled Y' + bias in channels [0, Cout), the skip in [Cout, Cout + Cs);
* backward: ``upcat_bwd`` turns d(cat) into dY' (pixel-unshuffled bilinear adjoint, a deterministic gather) and the
  dense skip gradient in one launch; dX = dY' Wr^T and dWr = X^T dY' on the same tall-skinny kernels (the weight
  gradient split over pixel chunks with fp32 partials, deterministic); the bias gradient is the channel
  sum of dY' (the bilinear weights of every output pixel sum to one).

``up_concat(up, x, skip)`` takes the fused path for an ``nn.ConvTranspose2d(Cin, Cout, 2, 2)`` on channels-last GPU
tensors (bf16, or fp32 under bf16 autocast) with Cout, Cs % 8 == 0 and a resize ratio within [0.5, 2]; anything else
runs the three-op reference sequence.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from .conv import _main_grad_cl, bias_grad

def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _compute_dtype(x: torch.Tensor) -> torch.dtype:
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


def up_concat_native_ok(up: nn.Module, x: torch.Tensor, skip: torch.Tensor) -> bool:
    if not (isinstance(up, nn.ConvTranspose2d) and _pair(up.kernel_size) == (2, 2) and _pair(up.stride) == (2, 2)
            and _pair(up.padding) == (0, 0) and _pair(up.output_padding) == (0, 0) and _pair(up.dilation) == (1, 1)
            and up.groups == 1):
        return False
    if not (x.is_cuda and skip.is_cuda and x.dim() == 4 and skip.dim() == 4 and _lib.use_native(x)):
        return False
    dt = _compute_dtype(x)
    if dt != torch.bfloat16 or skip.dtype != dt:
        return False
    n, _, h, w = x.shape
    co, cs, ho, wo = up.out_channels, skip.shape[1], skip.shape[2], skip.shape[3]
    return (skip.shape[0] == n and co % 8 == 0 and cs % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and skip.is_contiguous(memory_format=torch.channels_last) and skip.data_ptr() % 16 == 0
            and h <= ho <= 4 * h and w <= wo <= 4 * w)


def _tall_skinny_ok(cin: int, co: int) -> bool:
    return cin % 64 == 0 and (4 * co) % 64 == 0


class _Params:
    """The module's parameters behind a non-tensor argument (autograd does not track it): the backward writes their
    gradients straight into the engine's buckets (``main_grad``) instead of returning them."""

    __slots__ = ("weight", "bias")

    def __init__(self, weight, bias):
        self.weight, self.bias = weight, bias


class _UpConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, skip, params=None, bn_slot=None, skip_slot=None):
        n, cin, h, w = x.shape
        co = weight.shape[1]
        x2 = x.permute(0, 2, 3, 1).reshape(n * h * w, cin)          # channels-last: a view
        wr = weight.permute(0, 2, 3, 1).reshape(cin, 4 * co)        # (ci) x (i, j, co)
        ts = _tall_skinny_ok(cin, co)
        wrt = wr.t().contiguous() if ts else None                   # [(i, j, co), ci]
        # the [pixels, Cin] x [Cin, 4 Cout] GEMM on the tall-skinny kernels of csrc/conv1x1.hip when the channel
        # counts allow (they are written for M >> N, K), hipBLASLt otherwise
        y2 = _lib.ops().ts_gemm_nt(x2, wrt) if ts else torch.matmul(x2, wr)
        out = _lib.ops().upcat_fwd(y2, bias, skip, h, w)
        ctx.save_for_backward(x2, wr)
        ctx.dims = (n, cin, h, w, co)
        ctx.has_bias = bias is not None
        ctx.ts = ts
        ctx.params = params
        ctx.bn_slot = bn_slot
        # the skip's other consumer (the encoder's max pooling, ops.pool.SkipGradSlot) adds its gradient from d(concat)
        ctx.skip_slot = skip_slot if (skip_slot is not None and skip_slot.pool) else None
        if ctx.skip_slot is not None:
            skip_slot.armed = True
        return out

    @staticmethod
    def backward(ctx, dcat):
        x2, wr = ctx.saved_tensors
        n, cin, h, w, co = ctx.dims
        dcat = dcat.contiguous(memory_format=torch.channels_last)
        ss = ctx.skip_slot
        dy2, dskip = _lib.ops().upcat_bwd(dcat, h, w, co, ss is None)
        if ss is not None:
            ss.t, ss.off, dskip = dcat, co, None
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            bn = ctx.bn_slot   # x is a BatchNorm + ReLU output consumed only here: its reduction in this epilogue
            bn = bn if (bn is not None and ctx.ts and bn.usable(n * h * w, cin)) else None
            if bn is not None:
                dx2 = bn.launch(dy2, wr)
            else:
                dx2 = _lib.ops().ts_gemm_nt(dy2, wr) if ctx.ts else torch.matmul(dy2, wr.t())
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
            if bn is not None:
                bn.mark(dx)
        prm = ctx.params
        if ctx.needs_input_grad[1]:
            # a channels-last ConvTranspose2d weight [ci, co, 2, 2] is laid out as [ci, (i, j, co)] = dWr: the engine's
            # bucket view takes the weight-gradient kernel's output directly (no fp32 copy, permute or accumulate)
            mg = _main_grad_cl(prm.weight, cin, 4 * co) if (ctx.ts and prm is not None) else None
            if mg is not None:
                w = prm.weight
                _lib.ops().ts_gemm_tn_(mg, x2, dy2, bool(getattr(w, "_dph_accum", False)))
                w._dph_accum = True
                w._dph_grad_ready()
            else:
                if ctx.ts:   # dWr[ci, (i, j, co)] = X^T dY' over all pixels (split-pixel kernel, deterministic)
                    dwr = torch.empty((cin, 4 * co), device=x2.device, dtype=torch.float32)
                    _lib.ops().ts_gemm_tn_(dwr, x2, dy2, False)
                    dwr = dwr.to(x2.dtype)
                else:
                    dwr = torch.matmul(x2.t(), dy2)
                dw = dwr.view(cin, 2, 2, co).permute(0, 3, 1, 2).contiguous()
        if ctx.has_bias and ctx.needs_input_grad[2]:
            # straight into the bias's bucket view when the engine owns it (bias_grad), else returned in fp32
            db = bias_grad(prm.bias if prm is not None else None, dy2.view(-1, co), torch.float32)
        return dx, dw, db, dskip, None, None, None


def up_concat_reference(up: nn.Module, x: torch.Tensor, skip: torch.Tensor) -> torch.Tensor:
    """The reference sequence: transposed convolution, bilinear resize to the skip size if needed, concat."""
    u = up(x)
    if tuple(u.shape[2:]) != tuple(skip.shape[2:]):
        u = F.interpolate(u, size=skip.shape[2:], mode="bilinear", align_corners=False)
    return torch.cat([u, skip], dim=1)


def up_concat(up: nn.Module, x: torch.Tensor, skip: torch.Tensor, bn_slot=None, skip_slot=None) -> torch.Tensor:
    """``cat([resize(up(x), skip.shape[2:]), skip], 1)`` -- fused on the GPU when eligible.  ``bn_slot``
    (ops.conv.BnGradSlot): x is a BatchNorm + ReLU output consumed only here; its backward reduction then runs in the
    input-gradient GEMM's epilogue.  ``skip_slot`` (ops.pool.SkipGradSlot): the skip's gradient goes to its max
    pooling's backward instead of being copied out of d(concat)."""
    if not up_concat_native_ok(up, x, skip):
        return up_concat_reference(up, x, skip)
    dt = torch.bfloat16
    wt = up.weight if up.weight.dtype == dt else up.weight.to(dt)
    b = up.bias
    if b is not None and b.dtype != torch.float32:
        b = b.float()
    # the parameters themselves for the direct bucket writes -- only when the GEMM operand is the weight itself
    prm = _Params(up.weight, up.bias) if wt is up.weight and os.environ.get("DPH_UPCAT_DIRECT", "1") != "0" else None
    with torch.autocast("cuda", enabled=False):
        return _UpConcatFn.apply(x if x.dtype == dt else x.to(dt), wt, b, skip, prm,
                                 bn_slot if x.dtype == dt else None, skip_slot)
