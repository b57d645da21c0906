"""Async tensor parallelism: sequence-parallel collectives pipelined against the projection GEMMs.

Under Megatron-SP (parallel/tensor_parallel.py) every column-parallel projection is ``all_gather_seq(x) @ W^T`` and
every row-parallel one ``reduce_scatter_seq(x @ W^T)`` (2 all-gathers + 2 reduce-scatters of
[T, D] per layer and pass).  Run naively the GEMM waits for the whole collective and vice versa.  Here each
collective is split into ``chunks`` micro-collectives along the local sequence and all of them are issued up front
(async, on RCCL's stream); the compute stream waits for micro-collective i only before GEMM i, so GEMM i overlaps
collective i+1 (forward and backward, both directions):

    AG x GEMM (column-parallel):  y = AG(x) W^T    fwd: AG_i -> GEMM_i           bwd: GEMM_i -> RS_i (dx), one dW GEMM
    GEMM x RS (row-parallel):     y = RS(x W^T)    fwd: GEMM_i -> RS_i           bwd: AG_i -> GEMM_i (dx), one dW GEMM

Every micro-collective is a full RCCL all-gather / reduce-scatter over the TP group -- on the fully connected xGMI
mesh RCCL drives several links per collective, which a hand-rolled send/recv ring (one link per step) would not --
and the micro-chunks stay large (T D / (tp k) elements) so each keeps its plateau bandwidth.  The gathered
activations needed for dW are kept chunk-major ([k, tp, B, m, D]) so dW is ONE GEMM over all tokens, routed into the
data-parallel engine's flat gradient buffer when present (parallel/linear.py weight_grad).

Equivalent math to parallel/tensor_parallel.py's SP layers (gloo parity tests: tests/test_dist_llama.py::test_async_tp_*).  The
reference has no async-TP (its SP plan is plain DTensor redistribution, fsdp_tp/fsdp_tp_example.py:146-177).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .linear import weight_grad


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _chunks_for(seq_local: int, chunks: int) -> int:
    k = max(1, min(chunks, seq_local))
    while seq_local % k:
        k -= 1
    return k


def _ag_async(x: torch.Tensor, group, out: torch.Tensor | None = None):
    """all-gather of a contiguous [B, m, D] micro-chunk -> ([P, B, m, D] buffer, work); ``out`` (contiguous
    [P * B, m, D]) lets the caller gather straight into a slot of a larger buffer."""
    P = _ws(group)
    if out is None:
        out = torch.empty((P * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)   # dim-0 concatenation
    work = dist.all_gather_into_tensor(out, x, group=group, async_op=True)
    return out.view(P, *x.shape), work


def _rs_async(x: torch.Tensor, group, out: torch.Tensor | None = None):
    """reduce-scatter of a contiguous [P, B, m, D] partial -> ([B, m, D] buffer, work); ``out`` may be a contiguous
    slot of the caller's output (no concatenation afterwards)."""
    if out is None:
        out = torch.empty(x.shape[1:], dtype=x.dtype, device=x.device)
    inp = x.reshape(x.shape[0] * x.shape[1], *x.shape[2:])                              # dim-0 concatenation
    return out, dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group, async_op=True)


def _chunk_major(t: torch.Tensor, P: int, k: int) -> torch.Tensor:
    """[B, S, X] (S = P * k * m, rank-major sequence) -> contiguous [k, P, B, m, X]."""
    B, S, X = t.shape
    return t.reshape(B, P, k, S // (P * k), X).permute(2, 1, 0, 3, 4).contiguous()


def _seq_major(t: torch.Tensor) -> torch.Tensor:
    """[k, P, B, m, X] -> [B, S, X] (inverse of _chunk_major)."""
    k, P, B, m, X = t.shape
    return t.permute(2, 1, 0, 3, 4).reshape(B, P * k * m, X)


def _k_major(w: torch.Tensor, transpose_w: bool) -> torch.Tensor:
    """The K-contiguous [N, K] operand of ``x @ op(w)`` (op(w) = w^T: w itself; op(w) = w: its transpose, made ONCE per
    call -- HIP tile transpose on the GPU -- instead of once per micro-GEMM; hipBLASLt prefers this layout,
    parallel/linear.py _dgrad)."""
    if transpose_w:
        return w
    if w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous() and w.shape[0] % 8 == 0 \
            and w.shape[1] % 8 == 0:
        from ..ops import _lib

        if not _lib.reference_mode():
            return _lib.ops().transpose2d(w)
    return w.t().contiguous()


def _ag_matmul(x: torch.Tensor, w: torch.Tensor, group, k: int, transpose_w: bool):
    """AG(x) @ op(w) with k pipelined micro all-gathers; x [B, Sl, D].  Returns (y [B, S, N], gathered [k,P,B,m,D]).

    The micro all-gathers land in slots of ONE chunk-major buffer (kept for the weight gradient: no stack); each
    micro-GEMM is one 2-D GEMM whose [P, B, m, N] result is copied once into its rank-major sequence rows (overlapping
    the next micro all-gather).  A strided-batched GEMM writing those rows directly would need the weight broadcast at
    batch stride 0, which hipBLASLt on this stack rejects (parallel/linear.py _mm2d)."""
    B, Sl, D = x.shape
    P = _ws(group)
    m = Sl // k
    xg = torch.empty((k, P * B, m, D), dtype=x.dtype, device=x.device)
    pend = [_ag_async(x[:, i * m:(i + 1) * m].contiguous(), group, xg[i]) for i in range(k)]
    wk = _k_major(w, transpose_w)                                          # [N, D]
    N = wk.shape[0]
    y = torch.empty((B, P * Sl, N), dtype=x.dtype, device=x.device)
    yv = y.view(B, P, k, m, N)
    for i, (g, work) in enumerate(pend):
        work.wait()
        yi = torch.mm(g.reshape(-1, D), wk.t()).view(P, B, m, N)   # one 2-D GEMM (no batch-stride-0 broadcast)
        yv[:, :, i].copy_(yi.permute(1, 0, 2, 3))                   # [P, B, m, N] -> rank-major sequence order
    return y, xg.view(k, P, B, m, D)


def _matmul_rs(x_cm: torch.Tensor, w: torch.Tensor, group, transpose_w: bool) -> torch.Tensor:
    """RS(x @ op(w)) with the GEMM of micro-chunk i+1 overlapping the reduce-scatter of i; x_cm [k, P, B, m, F]
    chunk-major.  Returns [B, Sl, N] (this rank's sequence shard); with one sequence per rank (B = 1) the micro
    reduce-scatters write straight into their slice of it."""
    k, _, B, m, _ = x_cm.shape
    wk = _k_major(w, transpose_w)
    N = wk.shape[0]
    y = torch.empty((B, k * m, N), dtype=x_cm.dtype, device=x_cm.device) if B == 1 else None
    pend = []
    for i in range(k):
        part = torch.mm(x_cm[i].reshape(-1, x_cm.shape[-1]), wk.t()).view(*x_cm.shape[1:-1], N)
        pend.append(_rs_async(part, group, y[:, i * m:(i + 1) * m] if y is not None else None))
    outs = []
    for o, work in pend:
        work.wait()
        outs.append(o)
    return y if y is not None else torch.cat(outs, 1)


class _AGMatmulFn(torch.autograd.Function):
    """Column-parallel projection with a sequence-sharded input: y = AG_seq(x) W^T (+ b)."""

    @staticmethod
    def forward(ctx, x, w, b, group, chunks):
        k = _chunks_for(x.shape[1], chunks)
        y, xg = _ag_matmul(x.contiguous(), w, group, k, transpose_w=True)
        if b is not None:
            y = y + b
        ctx.save_for_backward(xg, w)
        ctx.group, ctx.k, ctx.has_bias = group, k, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xg, w = ctx.saved_tensors
        P, k = _ws(ctx.group), ctx.k
        dy_cm = _chunk_major(dy.contiguous(), P, k)                           # [k, P, B, m, N]
        dx = _matmul_rs(dy_cm, w, ctx.group, transpose_w=False) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            gw = weight_grad(w, dy_cm.reshape(-1, dy_cm.shape[-1]), xg.reshape(-1, xg.shape[-1]))
        gb = dy.reshape(-1, dy.shape[-1]).sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, gw, gb, None, None


class _MatmulRSFn(torch.autograd.Function):
    """Row-parallel projection producing a sequence-sharded output: y = RS_seq(x W^T); x [B, S, F_local]."""

    @staticmethod
    def forward(ctx, x, w, group, chunks):
        P = _ws(group)
        k = _chunks_for(x.shape[1] // P, chunks)
        x_cm = _chunk_major(x.contiguous(), P, k)                             # [k, P, B, m, F]
        y = _matmul_rs(x_cm, w, group, transpose_w=True)
        ctx.save_for_backward(x_cm, w)
        ctx.group, ctx.k = group, k
        return y

    @staticmethod
    def backward(ctx, dy):
        x_cm, w = ctx.saved_tensors
        dyc = dy.contiguous()
        dx, dyg = _ag_matmul(dyc, w, ctx.group, ctx.k, transpose_w=False)   # dyg [k, P, B, m, D] chunk-major
        gw = None
        if ctx.needs_input_grad[1]:
            gw = weight_grad(w, dyg.reshape(-1, dyg.shape[-1]), x_cm.reshape(-1, x_cm.shape[-1]))
        return (dx if ctx.needs_input_grad[0] else None), gw, None, None


def ag_matmul(x, w, b, group, chunks: int = 2):
    """y = all_gather_seq(x) @ w^T (+ b), x [B, S/tp, D] -> y [B, S, N_local]."""
    if _ws(group) == 1:
        return torch.nn.functional.linear(x, w, b)
    return _AGMatmulFn.apply(x, w, b, group, chunks)


def matmul_reduce_scatter(x, w, group, chunks: int = 2):
    """y = reduce_scatter_seq(x @ w^T), x [B, S, F_local] -> y [B, S/tp, D]."""
    if _ws(group) == 1:
        return torch.nn.functional.linear(x, w)
    return _MatmulRSFn.apply(x, w, group, chunks)
