"""Autograd-aware collectives (the conjugate pairs every model-parallel layer is built from).

Reference capability: the implicit DTensor redistributions of the TP/SP plan (fsdp_tp/fsdp_tp_example.py:142-184,
SURVEY.md C6-C11) and the doc-only Ulysses all-to-all / ring P2P (docs/guide/08_sequence_parallel.md).
Here each redistribution is one explicit RCCL call with its exact adjoint in backward:

    copy_to_group          fwd identity            bwd all-reduce          (Megatron "f")
    reduce_from_group      fwd all-reduce          bwd identity            (Megatron "g")
    gather_along_dim       fwd all-gather(dim)     bwd reduce-scatter(dim) (SP: Shard(1) -> Replicate)
    reduce_scatter_along   fwd reduce-scatter(dim) bwd all-gather(dim)     (SP: Partial -> Shard(1))
    split_along_dim        fwd take local chunk    bwd all-gather(dim)
    all_to_all_4d          fwd all-to-all          bwd inverse all-to-all  (Ulysses head<->sequence)

All collectives run on contiguous buffers (a transpose+contiguous at most) so RCCL moves one large
message per call; on gloo (CPU tests) the same code runs unchanged.

Sequence parallelism shards TOKENS, not the sequence dimension (``dim=TOKENS``).  An activation [B, S, D] is the
contiguous token matrix [B S, D]; rank r holds its share of the flat tokens and presents it as [B, S / tp, D].  Only
token-wise work (norms, residual adds) runs on the shard, so which tokens a rank holds is free, and choosing whole
runs of the flat order makes every gather / reduce-scatter a dim-0 collective on contiguous memory: no transpose
before it and no non-contiguous view after it (dim-1 sharding of [B, S, D] cost one full-size copy per collective
and another in the consumer -- 92 ms of a TP = 8 Llama-2-7B rank's 238 ms step, profiles/r5/tp_rank/).  With
``set_sp_chunks(group, k)`` (async TP) the flat tokens are dealt in k rounds of tp runs, so the k micro-collectives of
parallel/async_tp.py each fill one contiguous slice of the gathered tensor.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .custom_allreduce import use_custom as _use_custom


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


# ------------------------------------------------------------------------------------------- raw helpers
TOKENS = "tokens"      # the ``dim`` of a token-sharded (sequence-parallel) activation, see the module docstring
_SP_CHUNKS: dict = {}  # group key -> k (rounds of the token deal; 1 = one contiguous run per rank)


def _gkey(group):
    return id(group) if group is not None else "world"


def set_sp_chunks(group, k: int) -> None:
    """Token layout of ``group``'s sequence-parallel activations: k rounds (async TP's micro-collective count)."""
    _SP_CHUNKS[_gkey(group)] = max(1, int(k))


def sp_chunks(group, n_local: int = 0) -> int:
    """Rounds of the token deal for a shard of ``n_local`` tokens: the configured k, or its largest divisor of
    n_local (a function of (k, n_local) only, so every collective of a step -- all see the same token count -- and
    every rank agree on the layout)."""
    k = _SP_CHUNKS.get(_gkey(group), 1)
    if n_local > 0:
        k = max(1, min(k, n_local))
        while n_local % k:
            k -= 1
    return k


def _tok_shape(x: torch.Tensor, factor_num: int, factor_den: int = 1):
    """Shape of the gathered / scattered token tensor: [B, S, D] scales S (dim 1), [T, D] scales T (dim 0).  The
    TOKENS layout deals flattened tokens, so only token-wise ops may run on the shard (tensor_parallel.py)."""
    assert x.dim() in (2, 3), f"token-sharded tensors are [B, S, D] or [T, D], got {list(x.shape)}"
    shp = list(x.shape)
    shp[-2] = shp[-2] * factor_num // factor_den
    return shp


def tok_all_gather(x: torch.Tensor, group) -> torch.Tensor:
    """[B, Sl, D] token shard -> [B, Sl * tp, D] (natural token order), k dim-0 all-gathers into contiguous slots."""
    ws = _ws(group)
    if ws == 1:
        return x
    x = x.contiguous()
    d = x.shape[-1]
    n = x.numel() // d
    k = sp_chunks(group, n)
    m = n // k
    out = torch.empty((ws * n, d), dtype=x.dtype, device=x.device)
    xv, ov = x.view(k, m, d), out.view(k, ws * m, d)
    for c in range(k):
        dist.all_gather_into_tensor(ov[c], xv[c], group=group)
    return out.view(_tok_shape(x, ws))


def tok_reduce_scatter(x: torch.Tensor, group) -> torch.Tensor:
    """[B, S, D] partial sums -> this rank's [B, S / tp, D] token shard, k dim-0 reduce-scatters of contiguous slots."""
    ws = _ws(group)
    if ws == 1:
        return x
    x = x.contiguous()
    d = x.shape[-1]
    t = x.numel() // d
    assert x.dim() in (2, 3), f"token-sharded tensors are [B, S, D] or [T, D], got {list(x.shape)}"
    assert x.shape[-2] % ws == 0, f"reduce_scatter: {x.shape[-2]} positions do not split over {ws} ranks"
    k = sp_chunks(group, t // ws)
    m = t // (ws * k)
    out = torch.empty((k * m, d), dtype=x.dtype, device=x.device)
    xv, ov = x.view(k, ws * m, d), out.view(k, m, d)
    for c in range(k):
        dist.reduce_scatter_tensor(ov[c], xv[c], op=dist.ReduceOp.SUM, group=group)
    return out.view(_tok_shape(x, 1, ws))


def tok_split(x: torch.Tensor, group) -> torch.Tensor:
    """This rank's token shard of a replicated [B, S, D] (no communication)."""
    ws = _ws(group)
    if ws == 1:
        return x
    r = _rank(group)
    x = x.contiguous()
    d = x.shape[-1]
    t = x.numel() // d
    assert x.shape[1] % ws == 0, f"split: {x.shape[1]} positions do not split over {ws} ranks"
    k = sp_chunks(group, t // ws)
    m = t // (ws * k)
    return x.view(k, ws, m, d)[:, r].contiguous().view(_tok_shape(x, 1, ws))


def all_gather_dim(x: torch.Tensor, dim, group) -> torch.Tensor:
    if dim == TOKENS:
        return tok_all_gather(x, group)
    ws = _ws(group)
    if ws == 1:
        return x
    x = x.contiguous()
    if dim == 0:
        out = torch.empty((ws * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    xt = x.movedim(dim, 0).contiguous()
    out = torch.empty((ws * xt.shape[0], *xt.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, xt, group=group)
    return out.movedim(0, dim)


def reduce_scatter_dim(x: torch.Tensor, dim, group) -> torch.Tensor:
    if dim == TOKENS:
        return tok_reduce_scatter(x, group)
    ws = _ws(group)
    if ws == 1:
        return x
    assert x.shape[dim] % ws == 0, f"reduce_scatter: dim {dim} size {x.shape[dim]} not divisible by {ws}"
    xt = x.movedim(dim, 0).contiguous()
    out = torch.empty((xt.shape[0] // ws, *xt.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, xt, op=dist.ReduceOp.SUM, group=group)
    return out.movedim(0, dim)


def split_dim(x: torch.Tensor, dim, group) -> torch.Tensor:
    if dim == TOKENS:
        return tok_split(x, group)
    ws = _ws(group)
    if ws == 1:
        return x
    assert x.shape[dim] % ws == 0, f"split: dim {dim} size {x.shape[dim]} not divisible by {ws}"
    return x.chunk(ws, dim=dim)[_rank(group)].contiguous()


def all_reduce_(x: torch.Tensor, group, op=dist.ReduceOp.SUM) -> torch.Tensor:
    """In-place all-reduce.  SUM messages up to the group's measured crossover (comm/custom_allreduce.py
    probe_crossover / set_policy; ``DPH_CUSTOM_ALLREDUCE=1`` forces it up to ``DPH_CUSTOM_ALLREDUCE_MAX_BYTES``) take
    the direct-peer-read xGMI kernel; everything else goes to RCCL."""
    if _ws(group) > 1:
        if op == dist.ReduceOp.SUM and x.is_cuda:
            car = _use_custom(x, group)
            if car is not None:
                car.all_reduce(x)
                return x
        dist.all_reduce(x, op=op, group=group)
    return x


# ------------------------------------------------------------------------------------------- autograd
class _CopyToGroup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        return all_reduce_(g.contiguous(), ctx.group), None


class _ReduceFromGroup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        return all_reduce_(x.contiguous().clone() if _ws(group) > 1 else x, group)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherDim(torch.autograd.Function):
    """all-gather; adjoint = reduce-scatter (downstream work is partitioned across the group, so each rank
    holds a PARTIAL gradient of the gathered tensor -- sequence parallelism)."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return all_gather_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_dim(g, ctx.dim, ctx.group), None, None


class _GatherDimReplicated(torch.autograd.Function):
    """all-gather; adjoint = take the local chunk (downstream work is REPLICATED on every rank, so each rank
    already holds the full gradient -- e.g. gathering TP output logits before a replicated loss)."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return all_gather_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return split_dim(g, ctx.dim, ctx.group), None, None


class _ReduceScatterDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return reduce_scatter_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return all_gather_dim(g, ctx.dim, ctx.group), None, None


class _SplitDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return split_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return all_gather_dim(g, ctx.dim, ctx.group), None, None


def copy_to_group(x, group):
    return _CopyToGroup.apply(x, group) if _ws(group) > 1 else x


def reduce_from_group(x, group):
    return _ReduceFromGroup.apply(x, group) if _ws(group) > 1 else x


def gather_along_dim(x, dim, group):
    return _GatherDim.apply(x, dim, group) if _ws(group) > 1 else x


def gather_replicated_along_dim(x, dim, group):
    return _GatherDimReplicated.apply(x, dim, group) if _ws(group) > 1 else x


def reduce_scatter_along_dim(x, dim, group):
    return _ReduceScatterDim.apply(x, dim, group) if _ws(group) > 1 else x


def split_along_dim(x, dim, group):
    return _SplitDim.apply(x, dim, group) if _ws(group) > 1 else x


# ------------------------------------------------------------------------------------------- all-to-all
def _a2a(x: torch.Tensor, scatter_dim: int, gather_dim: int, group) -> torch.Tensor:
    """Split ``x`` into world chunks along scatter_dim, exchange, concatenate along gather_dim.

    Two copies in all: the input is laid out once with the rank as the leading dimension (the exchange buffer of
    all_to_all_single) and the output once into the gathered layout -- no per-chunk copies, stack or cat."""
    ws = _ws(group)
    if ws == 1:
        return x
    # normalise negative dims first: unflatten / movedim / flatten below index the ORIGINAL rank of x, and the
    # unflattened tensor has one more dimension (-1 would name the chunk, not the rank, dimension)
    scatter_dim %= x.dim()
    gather_dim %= x.dim()
    n = x.shape[scatter_dim]
    assert n % ws == 0, f"all_to_all: dim {scatter_dim} ({n}) not divisible by the group size {ws}"
    inp = x.unflatten(scatter_dim, (ws, n // ws)).movedim(scatter_dim, 0).contiguous()
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=group)
    return out.movedim(0, gather_dim).flatten(gather_dim, gather_dim + 1)


def _pack_heads(qkv: torch.Tensor, nh: int, nkv: int, hd: int, ws: int) -> torch.Tensor:
    """[B, s, (nh + 2 nkv) hd] -> exchange buffer [P, B, s, (nh + 2 nkv) / P * hd]: rank j's slot holds ITS q / k / v
    head groups, packed [q_j | k_j | v_j] (one copy)."""
    b, s, _ = qkv.shape
    q = qkv[..., : nh * hd].view(b, s, ws, nh // ws * hd)
    k = qkv[..., nh * hd: (nh + nkv) * hd].view(b, s, ws, nkv // ws * hd)
    v = qkv[..., (nh + nkv) * hd:].view(b, s, ws, nkv // ws * hd)
    return torch.cat([q, k, v], -1).movedim(2, 0).contiguous()


def _unpack_heads(buf: torch.Tensor, nh: int, nkv: int, hd: int, ws: int) -> torch.Tensor:
    """Inverse of ``_pack_heads``: [P, B, s, packed_j] -> [B, s, (nh + 2 nkv) hd]."""
    t = buf.movedim(0, 2)                                        # [B, s, P, packed]
    q, k, v = t.split([nh // ws * hd, nkv // ws * hd, nkv // ws * hd], -1)
    return torch.cat([q.flatten(2), k.flatten(2), v.flatten(2)], -1)


class _UlyssesQKV(torch.autograd.Function):
    """Sequence-sharded packed qkv [B, S/P, (nh + 2 nkv) hd] -> head-sharded, full-sequence packed qkv
    [B, S, (nh + 2 nkv) / P * hd] in ONE all-to-all (instead of one per q / k / v plus a concatenation)."""

    @staticmethod
    def forward(ctx, qkv, nh, nkv, hd, group):
        ws = _ws(group)
        ctx.cfg = (nh, nkv, hd, group)
        inp = _pack_heads(qkv, nh, nkv, hd, ws)
        out = torch.empty_like(inp)
        dist.all_to_all_single(out, inp, group=group)
        return out.movedim(0, 1).flatten(1, 2)                   # [B, P * s, packed]

    @staticmethod
    def backward(ctx, g):
        nh, nkv, hd, group = ctx.cfg
        ws = _ws(group)
        b, S, packed = g.shape
        inp = g.reshape(b, ws, S // ws, packed).movedim(1, 0).contiguous()
        out = torch.empty_like(inp)
        dist.all_to_all_single(out, inp, group=group)
        return _unpack_heads(out, nh, nkv, hd, ws), None, None, None, None


def ulysses_qkv(qkv: torch.Tensor, nh: int, nkv: int, hd: int, group) -> torch.Tensor:
    if _ws(group) == 1:
        return qkv
    assert nh % _ws(group) == 0 and nkv % _ws(group) == 0, "Ulysses needs head counts divisible by the group size"
    return _UlyssesQKV.apply(qkv, nh, nkv, hd, group)


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scatter_dim, gather_dim, group):
        ctx.dims, ctx.group = (scatter_dim, gather_dim), group
        return _a2a(x, scatter_dim, gather_dim, group)

    @staticmethod
    def backward(ctx, g):
        sd, gd = ctx.dims
        return _a2a(g, gd, sd, ctx.group), None, None, None


def all_to_all(x, scatter_dim: int, gather_dim: int, group):
    return _AllToAll.apply(x, scatter_dim, gather_dim, group) if _ws(group) > 1 else x


# ------------------------------------------------------------------------------------------- reductions for loss-parallel
class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return all_reduce_(x.clone(), group)

    @staticmethod
    def backward(ctx, g):
        return g, None


def all_reduce_autograd_sum(x, group):
    """sum over ranks feeding a REPLICATED downstream (every rank computes the same loss): grad is identity."""
    return _AllReduceSum.apply(x, group) if _ws(group) > 1 else x


class _AllReducePartial(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return all_reduce_(x.clone(), group)

    @staticmethod
    def backward(ctx, g):
        return all_reduce_(g.contiguous().clone(), ctx.group), None


def all_reduce_sum_partitioned(x, group):
    """sum over ranks feeding PARTITIONED downstream work (each rank's loss covers its own shard, total loss =
    sum over ranks): the adjoint is again an all-reduce (e.g. batch statistics of a domain-sharded field)."""
    return _AllReducePartial.apply(x, group) if _ws(group) > 1 else x


def all_reduce_autograd_max(x, group):
    """max over ranks, treated as a constant (used for the numerically-stable softmax shift only)."""
    x = x.detach().clone()
    return all_reduce_(x, group, op=dist.ReduceOp.MAX)
