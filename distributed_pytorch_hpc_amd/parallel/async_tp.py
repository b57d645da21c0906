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
and the micro-chunks stay large (T D / (tp k) elements) so each keeps its plateau bandwidth.

Layout: the sequence-parallel activations are token-sharded with the tokens dealt in k rounds
(comm/functional.py TOKENS, ``set_sp_chunks(group, k)``): round c of every rank's shard is one contiguous run of m
tokens, and the k x tp runs in (round, rank) order are the natural token order.  So micro-collective c gathers into
(or reduce-scatters out of) ONE contiguous slice [c tp m, (c+1) tp m) of the full [T, D] activation, every
micro-GEMM reads and writes contiguous rows, and the gathered activations needed for dW are the full tensor in
natural order -- dW is ONE GEMM, routed into the data-parallel engine's flat gradient buffer when present
(parallel/linear.py weight_grad).  No permute / copy anywhere (the round-4 form reordered every micro-GEMM's rows and
made chunk-major copies of x and dy).

Equivalent math to parallel/tensor_parallel.py's SP layers (gloo parity tests: tests/test_dist_llama.py::test_async_tp_*).  The
reference has no async-TP (its SP plan is plain DTensor redistribution, fsdp_tp/fsdp_tp_example.py:146-177).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .linear import weight_grad


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rounds(group, n_local: int) -> int:
    from ..comm.functional import sp_chunks

    return sp_chunks(group, n_local)


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


def _ag_matmul(x2: torch.Tensor, w: torch.Tensor, group, k: int, transpose_w: bool):
    """AG(x) @ op(w) with k pipelined micro all-gathers; x2 = this rank's [n, D] token shard.  Returns
    (y [P n, N], gathered x [P n, D]), both in natural token order: round c's all-gather lands in rows
    [c P m, (c+1) P m) of the gathered buffer and its GEMM writes the same rows of y."""
    P = _ws(group)
    n, D = x2.shape
    m = n // k
    xg = torch.empty((P * n, D), dtype=x2.dtype, device=x2.device)
    xs, gs = x2.view(k, m, D), xg.view(k, P * m, D)
    pend = [dist.all_gather_into_tensor(gs[c], xs[c], group=group, async_op=True) for c in range(k)]
    wk = _k_major(w, transpose_w)                                          # [N, D]
    y = torch.empty((P * n, wk.shape[0]), dtype=x2.dtype, device=x2.device)
    ys = y.view(k, P * m, wk.shape[0])
    for c, work in enumerate(pend):
        work.wait()
        torch.mm(gs[c], wk.t(), out=ys[c])
    return y, xg


def _matmul_rs(x2: torch.Tensor, w: torch.Tensor, group, k: int, transpose_w: bool) -> torch.Tensor:
    """RS(x @ op(w)) with the GEMM of round c+1 overlapping the reduce-scatter of round c; x2 [P n, F] in natural
    token order.  Returns this rank's [n, N] token shard."""
    P = _ws(group)
    T, F = x2.shape
    m = T // (P * k)
    wk = _k_major(w, transpose_w)
    N = wk.shape[0]
    y = torch.empty((k * m, N), dtype=x2.dtype, device=x2.device)
    xs, ys = x2.view(k, P * m, F), y.view(k, m, N)
    pend = []
    for c in range(k):
        part = torch.mm(xs[c], wk.t())
        pend.append((part, dist.reduce_scatter_tensor(ys[c], part, op=dist.ReduceOp.SUM, group=group,
                                                      async_op=True)))
    for _, work in pend:
        work.wait()
    return y


class _AGMatmulFn(torch.autograd.Function):
    """Column-parallel projection with a token-sharded input: y = AG_tokens(x) W^T (+ b)."""

    @staticmethod
    def forward(ctx, x, w, b, group, k):
        P = _ws(group)
        x = x.contiguous()
        y, xg = _ag_matmul(x.view(-1, x.shape[-1]), w, group, k, transpose_w=True)
        if b is not None:
            y = y + b
        ctx.save_for_backward(xg, w)
        ctx.group, ctx.k, ctx.has_bias, ctx.xshape = group, k, b is not None, x.shape
        shp = list(x.shape)
        shp[1] *= P
        shp[-1] = y.shape[-1]
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        xg, w = ctx.saved_tensors
        dy2 = dy.contiguous().view(-1, dy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _matmul_rs(dy2, w, ctx.group, ctx.k, transpose_w=False).view(ctx.xshape)
        gw = weight_grad(w, dy2, xg) if ctx.needs_input_grad[1] else None
        gb = dy2.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, gw, gb, None, None


class _MatmulRSFn(torch.autograd.Function):
    """Row-parallel projection producing a token-sharded output: y = RS_tokens(x W^T); x [B, S, F_local]."""

    @staticmethod
    def forward(ctx, x, w, group, k):
        P = _ws(group)
        x = x.contiguous()
        x2 = x.view(-1, x.shape[-1])
        y = _matmul_rs(x2, w, group, k, transpose_w=True)
        ctx.save_for_backward(x2, w)
        ctx.group, ctx.k, ctx.xshape = group, k, x.shape
        shp = list(x.shape)
        shp[1] //= P
        shp[-1] = y.shape[-1]
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.contiguous().view(-1, dy.shape[-1])
        dx, dyg = _ag_matmul(dy2, w, ctx.group, ctx.k, transpose_w=False)   # dyg: the gathered dy, natural order
        gw = weight_grad(w, dyg, x2) if ctx.needs_input_grad[1] else None
        return (dx.view(ctx.xshape) if ctx.needs_input_grad[0] else None), gw, None, None


def ag_matmul(x, w, b, group):
    """y = all_gather_tokens(x) @ w^T (+ b), x [B, S/tp, D] -> y [B, S, N_local].  The micro-collective count is the
    group's token layout (comm.functional.sp_chunks), which every SP collective of the group shares; a layer's
    ``async_chunks`` assignment sets it (tensor_parallel._AsyncChunks)."""
    if _ws(group) == 1:
        return torch.nn.functional.linear(x, w, b)
    return _AGMatmulFn.apply(x, w, b, group, _rounds(group, x.numel() // x.shape[-1]))


def matmul_reduce_scatter(x, w, group):
    """y = reduce_scatter_tokens(x @ w^T), x [B, S, F_local] -> y [B, S/tp, D]."""
    if _ws(group) == 1:
        return torch.nn.functional.linear(x, w)
    return _MatmulRSFn.apply(x, w, group, _rounds(group, x.numel() // x.shape[-1] // _ws(group)))
