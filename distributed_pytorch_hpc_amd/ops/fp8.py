"""Opt-in FP8-GEMM training (MI355X: OCP e4m3 / e5m2 MFMA at twice the bf16 rate).

The projection GEMMs of a linear layer run on hipBLASLt's FP8 kernels (``torch._scaled_mm``) with per-tensor current
scaling; everything else (attention, norms, activations, optimizer, master weights, the LM head) stays bf16 / fp32:

    forward   Y  = X W^T       X e4m3 [T, K] (row-major), W e4m3 [N, K]
    dgrad     dX = dY W        dY e5m2 [T, N], W^T e4m3 [K, N]
    wgrad     dW = dY^T X      dY^T e5m2 [N, T], X^T e4m3 [K, T]   (written into the engine's gradient bucket)

``csrc/fp8.hip`` makes the quantised copies in two passes over the bf16 tensor (amax, then scale + convert, the
row-major and the transposed copy from one read); the forward saves X^T in fp8 (1 byte per element) for the weight
gradient instead of the bf16 X, and W^T in fp8 for the input gradient (the weight is quantised once per step).  Scales follow the usual recipe: scale = FMAX / amax, dequantisation amax / FMAX.

Enable with ``DPH_FP8=1``, ``set_fp8(True)`` or any example driver's ``--fp8`` (train/cli.py); exempt a layer with
``exempt(module)`` (the Llama LM head is exempt by construction, and the marker survives tensor-parallel sharding).  Shapes the quantiser does not tile (any dim not a multiple of 64) fall back to the bf16 path.
This mode is NOT the headline precision: ``bench.py`` reports it only with ``--fp8`` and labels the dtype.
"""
from __future__ import annotations

import os

import torch

from . import _lib

E4M3, E5M2 = 0, 1
_enabled = os.environ.get("DPH_FP8", "0") == "1"


def set_fp8(flag: bool) -> None:
    global _enabled
    _enabled = bool(flag)


def fp8_enabled() -> bool:
    return _enabled


def exempt(module: torch.nn.Module) -> torch.nn.Module:
    """Keep ``module``'s linear weights on the bf16 path."""
    for p in module.parameters():
        p._dph_fp8_exempt = True
    return module


def enable_for_llama(model) -> None:
    """FP8 GEMMs for every projection of a models.llama2.Transformer except the LM head."""
    set_fp8(True)
    exempt(model.output)


def quantize(x: torch.Tensor, fmt: int, rowmajor: bool = True, transposed: bool = False):
    """(x_fp8 [R, C] or None, x_fp8^T [C, R] or None, dequant scale) for contiguous bf16 [R, C] on the GPU."""
    y, yt, s = _lib.ops().fp8_quantize(x, fmt, rowmajor, transposed)
    return (y if rowmajor else None), (yt if transposed else None), s


def applicable(x: torch.Tensor, w: torch.Tensor) -> bool:
    """x [..., K] and w [N, K] take the FP8 path: enabled, not exempt, bf16 on the GPU, all GEMM dims multiples of 64."""
    if not _enabled or getattr(w, "_dph_fp8_exempt", False) or not x.is_cuda or _lib.reference_mode():
        return False
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or w.dim() != 2 or not w.is_contiguous():
        return False
    k = x.shape[-1]
    t = x.numel() // max(k, 1)
    return x.dim() >= 2 and t % 64 == 0 and k % 64 == 0 and w.shape[0] % 64 == 0 and w.shape[1] == k


class _FP8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        k = x.shape[-1]
        x2 = x.reshape(-1, k).contiguous()
        xq, xqt, sx = quantize(x2, E4M3, rowmajor=True, transposed=w.requires_grad)
        # both weight copies from one pass: W for this GEMM, W^T (kept for the input gradient) if x needs one
        wq, wtq, sw = quantize(w, E4M3, rowmajor=True, transposed=x.requires_grad)
        # the output is allocated in its final shape (not returned as a view: callers rotate q / k in place)
        y = x2.new_empty(*x.shape[:-1], w.shape[0])
        torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw, out_dtype=torch.bfloat16, out=y.view(-1, w.shape[0]))
        empty = x2.new_empty(0)
        ctx.save_for_backward(xqt if xqt is not None else empty, sx, w, wtq if wtq is not None else empty, sw)
        ctx.x_shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..parallel.linear import weight_grad_from

        xqt, sx, w, wtq, sw = ctx.saved_tensors
        n = w.shape[0]
        g2 = gy.reshape(-1, n).contiguous()
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gq, gqt, sg = quantize(g2, E5M2, rowmajor=need_x, transposed=need_w)
        gx = gw = None
        if need_x:
            gx = gq.new_empty(ctx.x_shape, dtype=torch.bfloat16)   # dX = dY (W^T)^T with W^T [K, N] from the forward
            torch._scaled_mm(gq, wtq.t(), scale_a=sg, scale_b=sw, out_dtype=torch.bfloat16,
                             out=gx.view(-1, ctx.x_shape[-1]))
        if need_w:
            gw = weight_grad_from(w, lambda out: torch._scaled_mm(gqt, xqt.t(), scale_a=sg, scale_b=sx,
                                                                  out_dtype=out.dtype if out is not None
                                                                  else torch.bfloat16, out=out))
        return gx, gw


def fp8_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _FP8LinearFn.apply(x, w)
