"""Fused Llama sub-blocks: the projection GEMMs carry the neighbouring element-wise work in their epilogues
(csrc/gemm_nt.hip), forward and backward.

* ``swiglu_mlp(x, w13, w2)`` -- the FeedForward ``w2(silu(w1 x) * w3 x)`` of fsdp_tp/llama2_model.py:262-267.
  Forward: ONE kernel writes the saved gate / up projection AND h = silu(gate) * up (no swiglu_fwd pass), then
  y = h W2^T.  Backward: the input gradient of w2 runs with the SwiGLU backward in its epilogue (dh never touches
  HBM; no swiglu_bwd pass), then the w13 input / weight gradients.
* ``qkv_rope_attention(x, wqkv, ...)`` -- the attention core of fsdp_tp/llama2_model.py:176-228 from the block input:
  the wqkv projection applies RoPE to q / k on its fp32 accumulators (no rope pass, one rounding), flash attention
  forward; backward = flash backward with the inverse rotation in its epilogues + the projection's gradients.

Weight gradients take the same route as every other linear layer of the framework (parallel/linear.py:
``weight_grad`` writes them straight into the data-parallel engine's bucket and notifies it), so the engines'
overlapped reduce-scatter / all-reduce see no difference.  The fused paths are taken for bf16 projections whose
shapes the kernel tiles (rows % 256, features % 8, K % 8 -- shapes off the 256 / 64 grid run its ragged edge tiles),
plain or tensor-parallel: a ColwiseParallelLinear w13 / wqkv with a RowwiseParallelLinear w2 / wo (Megatron pair,
fsdp_tp/fsdp_tp_example.py:165-176) runs the same fused local computation between the pair's sequence all-gather
(or copy-to-group) and reduce-scatter (or all-reduce) -- at tp = 8 the 7B shards (SwiGLU H = 1376, w2's K = 1376)
tile as edge tiles.  FP8 and async-TP (pipelined micro-collectives) keep the unfused modules.  ``DPH_FUSED_MLP=0`` / ``DPH_FUSED_QKV=1`` switch them (A/B runs); by default the MLP's
fusions are on and the QKV + RoPE one is off.
"""
from __future__ import annotations

import math
import os

import torch

from ..ops import _lib
from ..ops import fp8 as _fp8
from .linear import _dgrad, weight_grad

# DPH_FUSED_MLP: "1" = SwiGLU in the w13 GEMM epilogue AND dSwiGLU in w2's input-gradient epilogue; "bwd" = only the
# backward fusion (forward: library GEMM + swiglu_fwd); "0" = unfused modules.  Default "1": the backward fusion
# measured +0.4 % on the Llama-2-7B step (profiles/r3/ab_fused_mlp_bwd/); the forward fusion, -0.6 % with the register
# epilogue, is +0.2 % since the GEMM's epilogue goes through LDS (w13 + SwiGLU 4.15 ms vs 4.24 for the library GEMM +
# swiglu_fwd; 28 128 / 28 070 vs 28 095 / 27 996 tokens/s, profiles/r3/ab_fused_mlp_fwd_lds/).
_FUSED_MLP = os.environ.get("DPH_FUSED_MLP", "1")
_FUSED_MLP = False if _FUSED_MLP == "0" else ("bwd" if _FUSED_MLP == "bwd" else True)
# DPH_FUSED_QKV=1: RoPE in the wqkv GEMM's epilogue -- off: -0.4 % in-step on the lookahead NT variant
# (profiles/r3/ab_fused_qkv_v1/) and -0.5 % still with the LDS epilogue (27 954 / 27 914 vs 28 128 / 28 070,
# profiles/r3/ab_fused_mlp_fwd_lds/): the kernel's 0.97x on wqkv outweighs the saved rope pass
_FUSED_QKV = os.environ.get("DPH_FUSED_QKV", "0") != "0"
# DPH_GEMM_NT: which forward / input-gradient GEMMs run on the CDNA4 kernel instead of hipBLASLt:
# "fused" (default: only those with a fused epilogue), "all", or "0" (none -- also disables the fused paths)
_GEMM_NT = os.environ.get("DPH_GEMM_NT", "fused")


def set_enabled(mlp: bool | None = None, qkv: bool | None = None, gemm_nt: str | None = None):
    """Toggle the fused paths at run time (tests / A/B runs); returns the previous (mlp, qkv, gemm_nt)."""
    global _FUSED_MLP, _FUSED_QKV, _GEMM_NT
    old = (_FUSED_MLP, _FUSED_QKV, _GEMM_NT)
    if mlp is not None:
        _FUSED_MLP = mlp if mlp == "bwd" else bool(mlp)
    if qkv is not None:
        _FUSED_QKV = bool(qkv)
    if gemm_nt is not None:
        _GEMM_NT = gemm_nt
    return old


_TOKENS = "tokens"   # comm.functional.TOKENS (the sequence-parallel token sharding)


def _plain_weight(mod) -> bool:
    from torch import nn

    return isinstance(mod, nn.Linear) and mod.bias is None and not getattr(mod.weight, "_dph_tp", False)


def _tp_col(mod, allow_async: bool = False) -> bool:
    from .tensor_parallel import ColwiseParallelLinear

    return (isinstance(mod, ColwiseParallelLinear) and mod.bias is None and not mod.gather_output and
            mod.seq_dim == _TOKENS and (allow_async or not mod.async_chunks))


def _tp_row(mod, allow_async: bool = False) -> bool:
    from .tensor_parallel import RowwiseParallelLinear

    return (isinstance(mod, RowwiseParallelLinear) and mod.bias is None and mod.input_is_parallel and
            mod.seq_dim == _TOKENS and (allow_async or not mod.async_chunks))


def _tp_pair(col, row, allow_async: bool = False) -> bool:
    return (_tp_col(col, allow_async) and _tp_row(row, allow_async) and col.group is row.group and col.sp == row.sp
            and bool(col.async_chunks) == bool(row.async_chunks))


def _async_pair(col, row) -> bool:
    """Both halves of the MLP pipelined against their sequence-parallel collectives (parallel/async_tp.py)."""
    return _tp_pair(col, row, allow_async=True) and col.sp and bool(col.async_chunks) and _tp_world(col) > 1


def _tp_world(mod) -> int:
    import torch.distributed as dist

    return dist.get_world_size(mod.group) if dist.is_initialized() else 1


def _tp_input(col, x):
    """The column-parallel layer's input as its local GEMM sees it: sequence-gathered (SP) or copied to the group."""
    from ..comm import functional as cf

    return cf.gather_along_dim(x, cf.TOKENS, col.group) if col.sp else cf.copy_to_group(x, col.group)


def _tp_output(row, y):
    from ..comm import functional as cf

    return cf.reduce_scatter_along_dim(y, cf.TOKENS, row.group) if row.sp else cf.reduce_from_group(y, row.group)


def _nt_ok(rows: int, n: int, k: int) -> bool:
    """Shapes the CDNA4 NT kernel tiles (csrc/gemm_nt.hip gemm_nt_supported): rows % 256, N % 8, K % 8, 32-bit
    offsets."""
    return rows > 0 and rows % 256 == 0 and n % 8 == 0 and k % 8 == 0 and n * k * 2 < (1 << 31)


def _native_bf16(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts) and not _lib.reference_mode() and \
        _lib.use_native(ts[0])


def _rows_ok(t: torch.Tensor) -> bool:
    return t.stride(-1) == 1 and t.is_contiguous() and t.data_ptr() % 16 == 0


def nt_enabled() -> bool:
    """Every forward / input-gradient GEMM of the framework's linear layers on the CDNA4 NT kernel (DPH_GEMM_NT=all)."""
    return _GEMM_NT == "all"


def nt_matmul(a2: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a2 [M, K] @ b[N, K]^T on the CDNA4 kernel when enabled for all GEMMs and tileable, else hipBLASLt."""
    if _GEMM_NT == "all" and _native_bf16(a2, b) and _nt_ok(a2.shape[0], b.shape[0], a2.shape[1]) and \
            _rows_ok(a2) and b.is_contiguous():
        return _lib.ops().gemm_nt(a2, b)
    return torch.matmul(a2, b.t())


def _dgrad_nt(g2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dY W for a [N, K] weight: the library path of parallel/linear.py, or the CDNA4 kernel on W^T."""
    if _GEMM_NT == "all" and _native_bf16(g2, w) and _nt_ok(g2.shape[0], w.shape[1], w.shape[0]) and \
            _rows_ok(g2) and w.is_contiguous():
        return _lib.ops().gemm_nt(g2, _lib.ops().transpose2d(w))
    return _dgrad(g2, w)


# ---------------------------------------------------------------------------------------------- SwiGLU MLP
class _SwiGLUMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w13, w2, fused_fwd=True):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if fused_fwd:
            x13, h = _lib.ops().gemm_nt_swiglu(x2, w13)
        else:
            x13 = torch.matmul(x2, w13.t())
            h = _lib.ops().swiglu_fwd(x13)
        y = nt_matmul(h, w2)
        ctx.save_for_backward(x2, w13, x13, h, w2)
        ctx.shape = shape
        return y.view(*shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w13, x13, h, w2 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        gx = gw13 = gw2 = None
        # w2's input gradient with the SwiGLU backward fused: d13 = [dgate | dup] straight from dh's accumulators
        w2t = _lib.ops().transpose2d(w2)
        d13 = _lib.ops().gemm_nt_dswiglu(dy2, w2t, x13)
        del w2t
        if ctx.needs_input_grad[2]:
            gw2 = weight_grad(w2, dy2, h)
        if ctx.needs_input_grad[0]:
            gx = _dgrad_nt(d13, w13).view(ctx.shape)
        if ctx.needs_input_grad[1]:
            gw13 = weight_grad(w13, d13, x2)
        return gx, gw13, gw2, None


def swiglu_mlp_ok(x: torch.Tensor, w13_mod, w2_mod) -> bool:
    if not (_FUSED_MLP and _GEMM_NT != "0"):
        return False
    tp = _tp_pair(w13_mod, w2_mod, allow_async=True)
    if not (tp or (_plain_weight(w13_mod) and _plain_weight(w2_mod))):
        return False
    if _fp8.fp8_enabled() or not _native_bf16(x, w13_mod.weight, w2_mod.weight) or not _rows_ok(x):
        return False
    rows, k = x.numel() // x.shape[-1], x.shape[-1]
    if tp and w13_mod.sp:
        if x.dim() != 3:
            return False
        rows *= _tp_world(w13_mod)            # the local GEMMs see the sequence-gathered activations
        if _async_pair(w13_mod, w2_mod):      # ... one round of the token deal at a time
            from ..comm.functional import sp_chunks

            rows //= sp_chunks(w13_mod.group, x.numel() // x.shape[-1])
    h2 = w13_mod.weight.shape[0]
    h, d_out = h2 // 2, w2_mod.weight.shape[0]
    return (h2 % 2 == 0 and w2_mod.weight.shape[1] == h and _nt_ok(rows, h2, k) and _nt_ok(rows, d_out, h)
            and _nt_ok(rows, h, d_out) and w13_mod.weight.is_contiguous() and w2_mod.weight.is_contiguous())


class _SwiGLUMLPAsyncFn(torch.autograd.Function):
    """The fused tensor-parallel SwiGLU MLP with both sequence-parallel collectives pipelined (async TP): round c of
    the token deal is all-gathered while the fused w13 + SwiGLU GEMM of round c-1 runs, and the w2 GEMM of round c
    overlaps the reduce-scatter of round c-1.  Backward mirrors it (all-gather of dy feeding the fused w2-dgrad +
    SwiGLU-backward GEMM, w13 dgrad feeding the reduce-scatter of dx); the weight gradients are one GEMM each over all
    tokens (natural order, comm/functional.py TOKENS)."""

    @staticmethod
    def forward(ctx, x, w13, w2, group, k):
        import torch.distributed as dist

        P = dist.get_world_size(group)
        x = x.contiguous()
        d = x.shape[-1]
        n = x.numel() // d
        m = n // k
        x2 = x.view(n, d)
        xg = torch.empty((P * n, d), dtype=x.dtype, device=x.device)
        xs, gs = x2.view(k, m, d), xg.view(k, P * m, d)
        pend = [dist.all_gather_into_tensor(gs[c], xs[c], group=group, async_op=True) for c in range(k)]
        h2, hl, dout = w13.shape[0], w13.shape[0] // 2, w2.shape[0]
        x13 = torch.empty((P * n, h2), dtype=x.dtype, device=x.device)
        h = torch.empty((P * n, hl), dtype=x.dtype, device=x.device)
        x13s, hs = x13.view(k, P * m, h2), h.view(k, P * m, hl)
        y = torch.empty((n, dout), dtype=x.dtype, device=x.device)
        ys = y.view(k, m, dout)
        rs = []
        for c, work in enumerate(pend):
            work.wait()
            _lib.ops().gemm_nt_swiglu_into(gs[c], w13, x13s[c], hs[c])
            part = nt_matmul(hs[c], w2)
            rs.append((part, dist.reduce_scatter_tensor(ys[c], part, op=dist.ReduceOp.SUM, group=group,
                                                        async_op=True)))
        for _, work in rs:
            work.wait()
        ctx.save_for_backward(xg, w13, x13, h, w2)
        ctx.group, ctx.k, ctx.shape = group, k, x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist

        xg, w13, x13, h, w2 = ctx.saved_tensors
        group, k = ctx.group, ctx.k
        P = dist.get_world_size(group)
        dy = dy.contiguous()
        dout = dy.shape[-1]
        n = dy.numel() // dout
        m = n // k
        dyg = torch.empty((P * n, dout), dtype=dy.dtype, device=dy.device)
        dys, gs = dy.view(k, m, dout), dyg.view(k, P * m, dout)
        pend = [dist.all_gather_into_tensor(gs[c], dys[c], group=group, async_op=True) for c in range(k)]
        w2t = _lib.ops().transpose2d(w2)
        h2 = x13.shape[1]
        d13 = torch.empty((P * n, h2), dtype=dy.dtype, device=dy.device)
        d13s, x13s = d13.view(k, P * m, h2), x13.view(k, P * m, h2)
        d = xg.shape[1]
        dx = torch.empty((n, d), dtype=dy.dtype, device=dy.device)
        dxs = dx.view(k, m, d)
        rs = []
        for c, work in enumerate(pend):
            work.wait()
            _lib.ops().gemm_nt_dswiglu_into(gs[c], w2t, x13s[c], d13s[c])
            part = _dgrad_nt(d13s[c], w13)
            rs.append((part, dist.reduce_scatter_tensor(dxs[c], part, op=dist.ReduceOp.SUM, group=group,
                                                        async_op=True)))
        del w2t
        gw2 = weight_grad(w2, dyg, h) if ctx.needs_input_grad[2] else None
        gw13 = weight_grad(w13, d13, xg) if ctx.needs_input_grad[1] else None
        for _, work in rs:
            work.wait()
        return dx.view(ctx.shape), gw13, gw2, None, None


def swiglu_mlp(x: torch.Tensor, w13_mod, w2_mod) -> torch.Tensor:
    if _async_pair(w13_mod, w2_mod):
        from ..comm.functional import sp_chunks

        return _SwiGLUMLPAsyncFn.apply(x, w13_mod.weight, w2_mod.weight, w13_mod.group,
                                       sp_chunks(w13_mod.group, x.numel() // x.shape[-1]))
    if _tp_pair(w13_mod, w2_mod):
        # Megatron pair: the local fused MLP between the column layer's input collective and the row layer's output
        # collective (their autograd adjoints give the backward's reduce-scatter / all-gather)
        y = _SwiGLUMLPFn.apply(_tp_input(w13_mod, x), w13_mod.weight, w2_mod.weight, _FUSED_MLP is True)
        return _tp_output(w2_mod, y)
    return _SwiGLUMLPFn.apply(x, w13_mod.weight, w2_mod.weight, _FUSED_MLP is True)


# ---------------------------------------------------------------------------------------------- QKV + RoPE + attention
class _QKVRopeAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wqkv, cos, sin, nh, nkv, hd, pos_offset):
        b, s, k = x.shape
        x2 = x.reshape(-1, k)
        n_rot = (nh + nkv) * hd
        qkv = _lib.ops().gemm_nt_rope(x2, wqkv, cos, sin, s, hd, n_rot, pos_offset).view(b, s, -1)
        q = qkv[:, :, : nh * hd].view(b, s, nh, hd)
        kk = qkv[:, :, nh * hd: n_rot].view(b, s, nkv, hd)
        v = qkv[:, :, n_rot:].view(b, s, nkv, hd)
        scale = 1.0 / math.sqrt(hd)
        o, lse = _lib.ops().flash_attn_fwd(q, kk, v, scale, True, 0.0, 0)
        ctx.save_for_backward(x2, wqkv, qkv, o, lse, cos, sin)
        ctx.cfg = (nh, nkv, hd, scale, pos_offset, x.shape)
        return o.view(b, s, nh * hd)

    @staticmethod
    def backward(ctx, do):
        x2, wqkv, qkv, o, lse, cos, sin = ctx.saved_tensors
        nh, nkv, hd, scale, pos_offset, xshape = ctx.cfg
        b, s, _ = qkv.shape
        n_rot = (nh + nkv) * hd
        q = qkv[:, :, : nh * hd].view(b, s, nh, hd)
        k = qkv[:, :, nh * hd: n_rot].view(b, s, nkv, hd)
        v = qkv[:, :, n_rot:].view(b, s, nkv, hd)
        dqkv = torch.empty_like(qkv)
        dq = dqkv[:, :, : nh * hd].view(b, s, nh, hd)
        dk = dqkv[:, :, nh * hd: n_rot].view(b, s, nkv, hd)
        dv = dqkv[:, :, n_rot:].view(b, s, nkv, hd)
        # dq / dk come out rotated back by -theta: the gradient w.r.t. the projection's (pre-RoPE) output
        _lib.ops().flash_attn_bwd_into(do.reshape(b, s, nh, hd).contiguous(), q, k, v, o, lse, scale, True,
                                       dq, dk, dv, 0.0, 0, cos, sin, pos_offset)
        g2 = dqkv.view(b * s, -1)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = _dgrad_nt(g2, wqkv).view(xshape)
        if ctx.needs_input_grad[1]:
            gw = weight_grad(wqkv, g2, x2)
        return gx, gw, None, None, None, None, None, None


def qkv_rope_attention_ok(x: torch.Tensor, wqkv_mod, hd: int) -> bool:
    tp = _tp_col(wqkv_mod)
    if not (_FUSED_QKV and _GEMM_NT != "0" and (tp or _plain_weight(wqkv_mod))) or x.dim() != 3:
        return False
    if _fp8.fp8_enabled() or not _native_bf16(x, wqkv_mod.weight) or not _rows_ok(x):
        return False
    b, s, k = x.shape
    if tp and wqkv_mod.sp:
        s *= _tp_world(wqkv_mod)
    n = wqkv_mod.weight.shape[0]
    return _nt_ok(b * s, n, k) and hd in (64, 128) and wqkv_mod.weight.is_contiguous()


def qkv_rope_attention(x, wqkv_mod, cos, sin, n_heads: int, n_kv_heads: int, head_dim: int,
                       pos_offset: int = 0) -> torch.Tensor:
    """n_heads / n_kv_heads: the LOCAL head counts (tensor-parallel: this rank's heads of the column shard)."""
    if _tp_col(wqkv_mod):
        x = _tp_input(wqkv_mod, x)
    return _QKVRopeAttnFn.apply(x, wqkv_mod.weight, cos, sin, n_heads, n_kv_heads, head_dim, pos_offset)
