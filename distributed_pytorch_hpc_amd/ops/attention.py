"""Flash attention on CDNA4 (csrc/attention.hip forward, csrc/attention_bwd.hip backward) and the fused RoPE+attention core of the Llama block.

Layout convention is [B, S, H, D] (sequence-major, heads inner) so that q/k/v are plain strided VIEWS of
the fused QKV GEMM output [B, S, (Hq + 2 Hkv) * D] -- no transposes, no copies.  The reference calls
``F.scaled_dot_product_attention(q, k, v, is_causal=True)`` on [B, H, S, D] transposed tensors
(fsdp_tp/llama2_model.py:214-225).

Head dims 32/64/128 run natively; 16/48/96 are zero-padded to the next native size (exact: padding the
contraction dim with zeros leaves QK^T unchanged, padded V columns are sliced off).  Larger head dims
fall back to ATen SDPA with a one-time warning.

Attention dropout (``dropout_p > 0``, the pipeline transformer's nn.MultiheadAttention(dropout=0.1),
03_pipeline_training.py:57-58) runs in the same kernels: the keep mask of element (query, key) is a counter hash
of (seed, batch*head, query, key) regenerated in the backward kernels, never stored; ``dropout_mask`` rebuilds
it for tests.  The seed comes from torch's CPU generator (``torch.manual_seed`` makes runs reproducible).
"""
from __future__ import annotations

import math
import os
import warnings

import torch
import torch.nn.functional as F

from . import _lib
from .rope import rope_, rope_reference

_NATIVE_D = (32, 64, 128)
# inverse RoPE of dq / dk in the backward kernels' epilogue (the separate pass stays for non-native shapes)
_FUSED_ROPE_BWD = True
_warned = set()


def _padded_dim(d: int) -> int | None:
    for n in _NATIVE_D:
        if d <= n:
            return n
    return None


def attention_reference(q, k, v, causal=True, scale=None):
    """fp32-capable reference on [B, S, H, D] inputs (GQA by head repetition)."""
    hq, hk = q.shape[2], k.shape[2]
    if hq != hk:
        k = k.repeat_interleave(hq // hk, dim=2)
        v = v.repeat_interleave(hq // hk, dim=2)
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    sq, sk = q.shape[1], k.shape[1]
    if causal and sq != sk:
        # bottom-right aligned causal mask (query i sees keys j <= i + sk - sq)
        i = torch.arange(sq, device=q.device)[:, None]
        j = torch.arange(sk, device=q.device)[None, :]
        mask = j <= i + (sk - sq)
        o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, scale=scale)
    else:
        o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale)
    return o.transpose(1, 2)


def _pad_last(t: torch.Tensor, d: int) -> torch.Tensor:
    return F.pad(t, (0, d - t.shape[-1]))


def flash_fwd(q, k, v, scale: float, causal: bool, dropout_p: float = 0.0, seed: int = 0):
    """Raw native forward: returns (o [B,S,Hq,D] bf16, lse fp32 [B,Hq,S]).  No autograd."""
    return _lib.ops().flash_attn_fwd(q, k, v, scale, causal, dropout_p, seed)


def flash_bwd(do, q, k, v, o, lse, scale: float, causal: bool, dropout_p: float = 0.0, seed: int = 0):
    """Raw native backward: returns (dq, dk, dv)."""
    return _lib.ops().flash_attn_bwd(do.contiguous(), q, k, v, o, lse, scale, causal, dropout_p, seed)


_M32 = 0xFFFFFFFF


def _mix(x: torch.Tensor) -> torch.Tensor:
    """csrc/attention_common.h attn_mix on int64 tensors holding uint32 values."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_mask(b: int, h: int, sq: int, sk: int, dropout_p: float, seed: int, device=None) -> torch.Tensor:
    """The kernels' keep mask as a bool [B, H, Sq, Sk] tensor (reference / tests)."""
    bh = torch.arange(b * h, device=device, dtype=torch.int64).view(b, h, 1, 1)
    q = torch.arange(sq, device=device, dtype=torch.int64).view(1, 1, sq, 1)
    k = torch.arange(sk, device=device, dtype=torch.int64).view(1, 1, 1, sk)
    row = _mix((seed & _M32) ^ _mix((bh * 0x9E3779B1 + q * 0x85EBCA77) & _M32))
    hsh = _mix(row ^ ((k * 0xC2B2AE3D) & _M32))
    thr = min(int(dropout_p * 4294967296.0), 4294967040)
    return hsh >= thr


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, dropout_p=0.0, seed=0):
        o, lse = flash_fwd(q, k, v, scale, causal, dropout_p, seed)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale, ctx.dropout_p, ctx.seed = causal, scale, dropout_p, seed
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = flash_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal, ctx.dropout_p, ctx.seed)
        return dq, dk, dv, None, None, None, None


def _native_ok(q: torch.Tensor) -> bool:
    return q.dtype == torch.bfloat16 and _lib.use_native(q)


def _sdpa_dropout(q, k, v, causal, scale, dropout_p):
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    return F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale,
                                          dropout_p=dropout_p).transpose(1, 2)


def flash_attention(q, k, v, causal: bool = True, scale: float | None = None, dropout_p: float = 0.0,
                    seed: int | None = None) -> torch.Tensor:
    """softmax(q k^T * scale [+ causal mask]) v on [B, S, H, D] tensors (GQA: Hq % Hkv == 0), with attention
    dropout ``dropout_p`` (pass it only in training)."""
    d = q.shape[-1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    if dropout_p > 0.0 and not (_native_ok(q) and _padded_dim(d) is not None):
        return _sdpa_dropout(q, k, v, causal, scale, dropout_p)
    if not _native_ok(q):
        return attention_reference(q, k, v, causal, scale)
    dp = _padded_dim(d)
    if dp is None:
        if "bigD" not in _warned:
            warnings.warn(f"flash_attention: head_dim {d} > 128 uses ATen SDPA")
            _warned.add("bigD")
        return attention_reference(q, k, v, causal, scale)
    if dp != d:
        q, k, v = _pad_last(q, dp), _pad_last(k, dp), _pad_last(v, dp)
    q, k, v = (t if t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:3]) else t.contiguous()
               for t in (q, k, v))
    if dropout_p > 0.0 and seed is None:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    o = _FlashAttnFn.apply(q, k, v, causal, scale, float(dropout_p), int(seed or 0))
    return o[..., :d] if dp != d else o


class _RopeFlashAttnFn(torch.autograd.Function):
    """o = attention(rope(q), rope(k), v) with q/k/v strided views of the fused QKV output.

    RoPE is applied IN PLACE to the q/k parts of ``qkv`` (marked dirty); backward runs the flash
    backward with the inverse rotation of dq/dk fused into its epilogues and returns one packed d(qkv).
    """

    @staticmethod
    def forward(ctx, qkv, cos, sin, n_heads, n_kv_heads, head_dim, causal, scale, pos_offset):
        b, s, _ = qkv.shape
        qk = qkv[:, :, : (n_heads + n_kv_heads) * head_dim].view(b, s, n_heads + n_kv_heads, head_dim)
        rope_(qk, cos, sin, pos_offset, False)
        q = qkv[:, :, : n_heads * head_dim].view(b, s, n_heads, head_dim)
        k = qkv[:, :, n_heads * head_dim: (n_heads + n_kv_heads) * head_dim].view(b, s, n_kv_heads, head_dim)
        v = qkv[:, :, (n_heads + n_kv_heads) * head_dim:].view(b, s, n_kv_heads, head_dim)
        o, lse = flash_fwd(q, k, v, scale, causal)
        ctx.mark_dirty(qkv)
        # the second output (the in-place-rotated qkv) is normally unused: do not materialise a zero gradient
        # for it (a [B, S, (Hq+2Hkv)*hd] fill + add per layer otherwise)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(qkv, o, lse, cos, sin)
        ctx.cfg = (n_heads, n_kv_heads, head_dim, causal, scale, pos_offset)
        return o.view(b, s, n_heads * head_dim), qkv

    @staticmethod
    def backward(ctx, do, _dqkv_passthrough):
        qkv, o, lse, cos, sin = ctx.saved_tensors
        nh, nkv, hd, causal, scale, pos_offset = ctx.cfg
        b, s, _ = qkv.shape
        q = qkv[:, :, : nh * hd].view(b, s, nh, hd)
        k = qkv[:, :, nh * hd: (nh + nkv) * hd].view(b, s, nkv, hd)
        v = qkv[:, :, (nh + nkv) * hd:].view(b, s, nkv, hd)
        dqkv = torch.empty_like(qkv)
        dq = dqkv[:, :, : nh * hd].view(b, s, nh, hd)
        dk = dqkv[:, :, nh * hd: (nh + nkv) * hd].view(b, s, nkv, hd)
        dv = dqkv[:, :, (nh + nkv) * hd:].view(b, s, nkv, hd)
        if _FUSED_ROPE_BWD:
            # dq / dk leave the kernels already rotated back by -theta (RoPE's gradient, from the fp32 accumulators)
            _lib.ops().flash_attn_bwd_into(do.view(b, s, nh, hd).contiguous(), q, k, v, o, lse, scale, causal,
                                           dq, dk, dv, 0.0, 0, cos, sin, pos_offset)
        else:
            _lib.ops().flash_attn_bwd_into(do.view(b, s, nh, hd).contiguous(), q, k, v, o, lse, scale, causal,
                                           dq, dk, dv)
            rope_(dqkv[:, :, : (nh + nkv) * hd].view(b, s, nh + nkv, hd), cos, sin, pos_offset, True)
        if _dqkv_passthrough is not None:
            dqkv = dqkv + _dqkv_passthrough
        return dqkv, None, None, None, None, None, None, None, None


def rope_attention(qkv: torch.Tensor, cos, sin, n_heads: int, n_kv_heads: int, head_dim: int,
                   causal: bool = True, pos_offset: int = 0) -> torch.Tensor:
    """Fused RoPE + causal attention on a packed [B, S, (Hq + 2 Hkv) * hd] projection output.

    Returns [B, S, Hq * hd].
    """
    scale = 1.0 / math.sqrt(head_dim)
    b, s, _ = qkv.shape
    if _native_ok(qkv) and head_dim in _NATIVE_D and qkv.is_contiguous():
        o, _ = _RopeFlashAttnFn.apply(qkv, cos, sin, n_heads, n_kv_heads, head_dim, causal, scale, pos_offset)
        return o
    q = qkv[:, :, : n_heads * head_dim].view(b, s, n_heads, head_dim)
    k = qkv[:, :, n_heads * head_dim: (n_heads + n_kv_heads) * head_dim].view(b, s, n_kv_heads, head_dim)
    v = qkv[:, :, (n_heads + n_kv_heads) * head_dim:].view(b, s, n_kv_heads, head_dim)
    if qkv.is_cuda:
        from .rope import apply_rope

        q, k = apply_rope(q, cos, sin, pos_offset), apply_rope(k, cos, sin, pos_offset)
    else:
        q, k = rope_reference(q, cos, sin, pos_offset), rope_reference(k, cos, sin, pos_offset)
    o = flash_attention(q, k, v, causal, scale)
    return o.reshape(b, s, n_heads * head_dim)
