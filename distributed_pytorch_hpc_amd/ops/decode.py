"""Serving-path ops: KV-cache append (RoPE fused) and single-token decode attention (csrc/decode.hip).

The reference is training-only (fsdp_tp/llama2_model.py has no cache); these ops back ``models.llama2.KVCache`` and
``inference.Generator``.  Layout: the fused QKV projection output [B, S, (Hq + 2 Hkv) * D] (the same buffer the
training path rotates in place) and per-layer caches [B, Smax, Hkv, D]; ``pos`` is an int32 [B] device tensor with
the number of tokens already cached per sequence, so a decode step never needs the lengths on the host (HIP graphs).

GPU tensors run the HIP kernels (the extension must be present); CPU tensors run the PyTorch references below, which
are also the oracles of tests/test_decode_gpu.py.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .attention import attention_reference
from .rope import rope_reference


def _split(qkv: torch.Tensor, n_heads: int, n_kv_heads: int, head_dim: int):
    b, s, _ = qkv.shape
    q = qkv[:, :, : n_heads * head_dim].view(b, s, n_heads, head_dim)
    k = qkv[:, :, n_heads * head_dim: (n_heads + n_kv_heads) * head_dim].view(b, s, n_kv_heads, head_dim)
    v = qkv[:, :, (n_heads + n_kv_heads) * head_dim:].view(b, s, n_kv_heads, head_dim)
    return q, k, v


FP8_KV = torch.float8_e4m3fn
FP8_MAX = 448.0


def quantize_kv(x: torch.Tensor, scale: float) -> torch.Tensor:
    """bf16 keys / values -> OCP e4m3 cache entries (x / scale, saturated; torch's cast itself does not saturate)."""
    return (x.to(torch.bfloat16).float() / scale).clamp(-FP8_MAX, FP8_MAX).to(FP8_KV)


def dequantize_kv(c: torch.Tensor, scale: float, dtype: torch.dtype) -> torch.Tensor:
    return c if c.dtype != FP8_KV else (c.float() * scale).to(dtype)


def kv_append_reference(qkv, k_cache, v_cache, pos, cos, sin, n_heads: int, n_kv_heads: int,
                        kv_scale: float = 1.0) -> None:
    hd = k_cache.shape[-1]
    q, k, v = _split(qkv, n_heads, n_kv_heads, hd)
    s = qkv.shape[1]
    fp8 = k_cache.dtype == FP8_KV
    for b, p in enumerate(pos.tolist()):
        if p + s > k_cache.shape[1]:
            raise ValueError(f"kv cache overflow: sequence {b} at {p} + {s} > capacity {k_cache.shape[1]}")
        q[b:b + 1].copy_(rope_reference(q[b:b + 1], cos, sin, p))
        kr = rope_reference(k[b:b + 1], cos, sin, p)[0]
        k_cache[b, p:p + s].copy_(quantize_kv(kr, kv_scale) if fp8 else kr)
        v_cache[b, p:p + s].copy_(quantize_kv(v[b], kv_scale) if fp8 else v[b])


def kv_append_(qkv: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, pos: torch.Tensor, cos: torch.Tensor,
               sin: torch.Tensor, n_heads: int, n_kv_heads: int, kv_scale: float = 1.0) -> None:
    """Rotate q in place in ``qkv`` [B, S, (Hq + 2 Hkv) * D], write rotated k and v into the caches at positions
    pos[b] .. pos[b] + S - 1 (bf16, or OCP e4m3 holding value / kv_scale).  ``pos`` is not advanced (the caller
    does that once per model step)."""
    if _lib.use_native(qkv):
        _lib.ops().kv_append_(qkv, k_cache, v_cache, pos, cos, sin, n_heads, n_kv_heads, float(kv_scale))
        return
    kv_append_reference(qkv, k_cache, v_cache, pos, cos, sin, n_heads, n_kv_heads, kv_scale)


def decode_attention_reference(qkv, k_cache, v_cache, pos, n_heads: int, n_kv_heads: int, scale: float,
                               kv_scale: float = 1.0):
    hd = k_cache.shape[-1]
    q, _, _ = _split(qkv, n_heads, n_kv_heads, hd)
    outs = []
    for b, p in enumerate(pos.tolist()):
        n = p + 1
        kk = dequantize_kv(k_cache[b:b + 1, :n], kv_scale, torch.float32).float()
        vv = dequantize_kv(v_cache[b:b + 1, :n], kv_scale, torch.float32).float()
        outs.append(attention_reference(q[b:b + 1].float(), kk, vv, causal=False, scale=scale))
    return torch.cat(outs, 0).reshape(qkv.shape[0], n_heads * hd).to(qkv.dtype)


def decode_attention(qkv: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, pos: torch.Tensor, n_heads: int,
                     n_kv_heads: int, scale: float | None = None, max_len: int | None = None,
                     kv_scale: float = 1.0) -> torch.Tensor:
    """Attention of the single new token per sequence (qkv [B, 1, ...], already appended) over keys 0 .. pos[b];
    returns [B, Hq * D].  ``max_len`` bounds pos + 1 over the batch (default: the cache capacity, as in a captured
    graph); a tighter bound only launches fewer workgroups."""
    hd = k_cache.shape[-1]
    scale = 1.0 / math.sqrt(hd) if scale is None else scale
    if _lib.use_native(qkv):
        return _lib.ops().decode_attention(qkv, k_cache, v_cache, pos, n_heads, n_kv_heads, scale,
                                           int(max_len or k_cache.shape[1]), float(kv_scale))
    return decode_attention_reference(qkv, k_cache, v_cache, pos, n_heads, n_kv_heads, scale, kv_scale)


def skinny_ok(x: torch.Tensor, mod: torch.nn.Module) -> bool:
    """A bias-free nn.Linear call with decode-sized row count (<= 64) that the weight-streaming kernel covers.
    Modules with hooks (FSDP units gather their weights in them) keep the module call."""
    w = getattr(mod, "weight", None)
    if w is None or getattr(mod, "bias", None) is not None or mod._forward_hooks or mod._forward_pre_hooks:
        return False
    if not (x.is_cuda and w.is_cuda) or _lib.reference_mode() or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if w.dim() != 2 or not w.is_contiguous() or x.shape[-1] != w.shape[1] or x.stride(-1) != 1:
        return False
    k, n = w.shape[1], w.shape[0]
    m = x.numel() // max(k, 1)
    # 1-2 rows: the GEMV form (any N % 8, K % 8, K <= 16384).  3-16 rows: the MFMA form (4 waves x unroll 4) where it
    # measured faster than hipBLASLt (benchmarks/skinny_gemm_bench.py, profiles/serving/skinny_sweep/): every 7B
    # projection up to 4 rows, up to 8 rows below N = 24 576 (wqkv, w13), up to 16 rows at N <= 8192 (wo, w2: 1.5-2x);
    # the LM head from 8 rows and the wide projections from 16 rows stay on hipBLASLt's tiled reuse of x
    if m <= 2:
        return m >= 1 and n % 8 == 0 and k % 8 == 0 and k <= 16384
    if n % 16 or k % 128:
        return False
    return m <= 4 or (m <= 8 and n <= 24576) or (m <= 16 and n <= 8192)


def skinny_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T for at most 64 rows (decode): streams W once at HBM rate (csrc/decode.hip)."""
    return _lib.ops().skinny_linear(x, w)


def _plain(mod) -> bool:
    return not mod._forward_hooks and not mod._forward_pre_hooks


def fused_decode_ok(x: torch.Tensor, *mods) -> bool:
    """One decode row (batch 1) on the GPU with plain bias-free bf16 nn.Linear / norm modules: the producer-fused
    GEMV path (RMSNorm or SwiGLU computed inside the projection kernel) applies."""
    if not x.is_cuda or _lib.reference_mode() or x.dtype != torch.bfloat16 or x.numel() != x.shape[-1]:
        return False
    for m in mods:
        w = getattr(m, "weight", None)
        if w is None or not _plain(m) or getattr(m, "bias", None) is not None or w.dtype != torch.bfloat16:
            return False
        if w.dim() == 2 and type(m) is not torch.nn.Linear:   # tensor-parallel wrappers do collectives in forward
            return False
        if not w.is_contiguous() or (w.dim() == 2 and (w.shape[0] % 8 or w.shape[1] % 8 or w.shape[1] > 16384)):
            return False
    return True


def gemv_rmsnorm(x: torch.Tensor, res: torch.Tensor | None, norm_weight: torch.Tensor, eps: float, w: torch.Tensor):
    """(RMSNorm(x + res) * g) @ w^T for one row, the norm computed inside the GEMV kernel; returns (y, h = x + res)."""
    y, h = _lib.ops().gemv_rmsnorm(x, res, norm_weight, eps, w)
    return y, (x if res is None else h)


def gemv_swiglu(x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """(silu(gate) * up) @ w^T for 1-2 rows of the fused [gate | up] projection output."""
    return _lib.ops().gemv_swiglu(x2, w)
