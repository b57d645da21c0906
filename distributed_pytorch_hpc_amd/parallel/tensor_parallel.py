"""Tensor parallelism (Megatron 1-D) and sequence parallelism over an explicit TP process group.

Capability parity with the reference's DTensor plans -- ``parallelize_module`` with ``ColwiseParallel``,
``RowwiseParallel``, ``SequenceParallel`` and ``PrepareModuleInput`` (fsdp_tp/tensor_parallel_example.py:115-122,
scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:352-361, fsdp_tp/fsdp_tp_example.py:142-184) -- but every
layout change is one explicit RCCL collective with a hand-written adjoint (comm/functional.py) and the
parameters stay plain tensors (local shards), so the data-parallel engine, the fused optimizer and the
HIP kernels see ordinary contiguous buffers.

Styles (applied by ``parallelize_module(module, tp_group, plan)``):
  ColwiseParallel(sequence_parallel=False, gather_output=False, shard_fn=None)
      weight [out, in] -> rows out/tp.  Input: replicated (copy_to_group: grad all-reduced) or, with
      sequence_parallel, token-sharded and all-gathered (grad reduce-scattered).  The default SP layout is TOKENS
      (comm/functional.py): the [B, S/tp, D] shard is a view of k contiguous runs of the FLATTENED B*S tokens, not of
      batch rows, so the collectives move contiguous rank slots with no transposes.  Its contract: every module in
      the SP region must be token-wise (norms, projections, activations); anything per-sample or position-dependent
      (attention, RoPE) runs after the all-gather on the full sequence.
  RowwiseParallel(sequence_parallel=False, shard_fn=None)
      weight [out, in] -> columns in/tp.  Output: partial sums all-reduced, or reduce-scattered along the
      sequence (SP).  A bias is added once, after the reduction.
  VocabParallelEmbedding(sequence_parallel=False)
      table rows vocab/tp; out-of-shard ids give zero rows (HIP gather kernel), partial embeddings are
      all-reduced or reduce-scattered along the sequence (SP) -- the reference's
      RowwiseParallel(input_layouts=Replicate(), output_layouts=Shard(1)) on tok_embeddings.
  SequenceParallel()
      replicated weights of a per-token module (norms) that runs on a sequence shard; their gradients
      are all-reduced over the TP group (partial over the local tokens).

``parallelize_llama(model, tp_group, sequence_parallel=True, loss_parallel=True)`` applies the TorchTitan-style
plan of the reference (fsdp_tp_example.py:142-184) to models/llama2.Transformer, including the fused
wqkv / w13 projections (sharded per head / per half) and vocab-parallel cross-entropy ("loss parallel":
only [N] all-reduces instead of all-gathering [B, S, V] logits).
"""
from __future__ import annotations

import warnings

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch import nn

from .. import ops
from ..comm import functional as cf
from .async_tp import ag_matmul, matmul_reduce_scatter
from .linear import linear as _linear


def _ws(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group):
    return dist.get_rank(group) if dist.is_initialized() else 0


def shard_rows(w: torch.Tensor, group) -> torch.Tensor:
    ws, r = _ws(group), _rank(group)
    assert w.shape[0] % ws == 0, f"cannot shard {w.shape[0]} rows over {ws} ranks"
    return w.chunk(ws, 0)[r].contiguous()


def shard_cols(w: torch.Tensor, group) -> torch.Tensor:
    ws, r = _ws(group), _rank(group)
    assert w.shape[1] % ws == 0, f"cannot shard {w.shape[1]} columns over {ws} ranks"
    return w.chunk(ws, 1)[r].contiguous()


def shard_rows_grouped(w: torch.Tensor, sizes: list[int], group) -> torch.Tensor:
    """Row-shard each block of a row-concatenated fused weight separately (wqkv = [q; k; v], w13 = [w1; w3])."""
    parts = torch.split(w, sizes, 0)
    return torch.cat([shard_rows(p, group) for p in parts], 0).contiguous()


def _carry_flags(src: torch.Tensor, dst: torch.Tensor) -> None:
    """Per-parameter markers survive sharding (e.g. ops/fp8.py's exemption of the LM head)."""
    if getattr(src, "_dph_fp8_exempt", False):
        dst._dph_fp8_exempt = True


class ColwiseParallelLinear(nn.Module):
    def __init__(self, lin: nn.Linear, group, sequence_parallel: bool = False, gather_output: bool = False,
                 shard_fn: Optional[Callable] = None, seq_dim=cf.TOKENS):
        super().__init__()
        self.group, self.sp, self.gather_output, self.seq_dim = group, sequence_parallel, gather_output, seq_dim
        w = lin.weight.detach()
        self.weight = nn.Parameter(shard_fn(w, group) if shard_fn else shard_rows(w, group),
                                   requires_grad=lin.weight.requires_grad)
        _carry_flags(lin.weight, self.weight)
        self.bias = None
        if lin.bias is not None:
            self.bias = nn.Parameter(shard_rows(lin.bias.detach()[:, None], group)[:, 0].contiguous())
        self.in_features, self.out_features = lin.in_features, self.weight.shape[0]
        self.async_chunks = 0   # > 0: sequence all-gather pipelined against the GEMM (parallel/async_tp.py)

    async_chunks = property(lambda self: self._async_chunks, lambda self, k: _set_async_chunks(self, k))

    def forward(self, x):
        if self.sp and self.async_chunks and self.seq_dim == cf.TOKENS and x.dim() == 3 and _ws(self.group) > 1:
            y = ag_matmul(x, self.weight, self.bias, self.group)
        else:
            x = cf.gather_along_dim(x, self.seq_dim, self.group) if self.sp else cf.copy_to_group(x, self.group)
            y = _linear(x, self.weight, self.bias)
        if self.gather_output:
            y = cf.gather_replicated_along_dim(y, y.dim() - 1, self.group)
        return y


def _set_async_chunks(mod, k) -> None:
    """``layer.async_chunks = k`` (k > 0) pipelines the layer's SP collective in k micro-collectives.  The count is a
    property of the TP group's token layout (comm.functional.set_sp_chunks), shared by every SP collective of the
    group, so assigning it here sets the layout too -- a plan that sets ``async_chunks`` directly gets the overlap it
    asked for (advisor r5: the count used to be read from the layout only, which only parallelize_llama set)."""
    k = int(k)
    object.__setattr__(mod, "_async_chunks", k)
    if k > 0 and mod.sp:
        prev = cf.sp_chunks(mod.group)
        if prev not in (1, k):
            warnings.warn(f"async_chunks={k} replaces the TP group's SP layout of {prev} rounds for every layer of "
                          "the group", stacklevel=3)
        cf.set_sp_chunks(mod.group, k)


class RowwiseParallelLinear(nn.Module):
    def __init__(self, lin: nn.Linear, group, sequence_parallel: bool = False, shard_fn: Optional[Callable] = None,
                 input_is_parallel: bool = True, seq_dim=cf.TOKENS):
        super().__init__()
        self.group, self.sp, self.input_is_parallel, self.seq_dim = group, sequence_parallel, input_is_parallel, seq_dim
        w = lin.weight.detach()
        self.weight = nn.Parameter(shard_fn(w, group) if shard_fn else shard_cols(w, group),
                                   requires_grad=lin.weight.requires_grad)
        _carry_flags(lin.weight, self.weight)
        self.bias = nn.Parameter(lin.bias.detach().clone()) if lin.bias is not None else None
        self.in_features, self.out_features = self.weight.shape[1], lin.out_features
        self.async_chunks = 0   # > 0: GEMM pipelined against the sequence reduce-scatter (parallel/async_tp.py)

    async_chunks = property(lambda self: self._async_chunks, lambda self, k: _set_async_chunks(self, k))

    def forward(self, x):
        if not self.input_is_parallel:
            x = cf.split_along_dim(x, x.dim() - 1, self.group)
        if self.sp and self.async_chunks and self.seq_dim == cf.TOKENS and x.dim() == 3 and _ws(self.group) > 1:
            y = matmul_reduce_scatter(x, self.weight, self.group)
        else:
            y = _linear(x, self.weight, None)
            y = cf.reduce_scatter_along_dim(y, self.seq_dim, self.group) if self.sp else \
                cf.reduce_from_group(y, self.group)
        if self.bias is not None:
            y = y + self.bias
        return y


class VocabParallelEmbedding(nn.Module):
    def __init__(self, emb: nn.Embedding, group, sequence_parallel: bool = False, seq_dim=cf.TOKENS):
        super().__init__()
        self.group, self.sp, self.seq_dim = group, sequence_parallel, seq_dim
        ws, r = _ws(group), _rank(group)
        v = emb.weight.shape[0]
        assert v % ws == 0, f"vocab {v} not divisible by tp {ws}"
        self.vocab_start = r * (v // ws)
        self.weight = nn.Parameter(shard_rows(emb.weight.detach(), group))

    def forward(self, ids):
        y = ops.embedding(ids, self.weight, self.vocab_start)
        return cf.reduce_scatter_along_dim(y, self.seq_dim, self.group) if self.sp else cf.reduce_from_group(y, self.group)


def mark_sequence_parallel(module: nn.Module, group):
    """Replicated params of a module that runs on a sequence shard: their grads are partial over TP.  A
    data-parallel engine that owns them (parallel/data_parallel.py) completes ALL of them with one all-reduce per
    step after its own reduction (``_dph_tp_batched``); without an engine a backward hook all-reduces each one."""
    if _ws(group) == 1:
        return module
    for p in module.parameters(recurse=False):
        p._dph_sequence_parallel = True
        p._dph_sp_group = group
        p.register_hook(lambda g, grp=group, prm=p: g if getattr(prm, "_dph_tp_batched", False)
                        else cf.all_reduce_(g.contiguous().clone(), grp))
    return module


# ------------------------------------------------------------------------------------------- plan API
@dataclass
class ColwiseParallel:
    sequence_parallel: bool = False
    gather_output: bool = False
    shard_fn: Optional[Callable] = None

    def apply(self, mod, group):
        return ColwiseParallelLinear(mod, group, self.sequence_parallel, self.gather_output, self.shard_fn)


@dataclass
class RowwiseParallel:
    sequence_parallel: bool = False
    shard_fn: Optional[Callable] = None
    input_is_parallel: bool = True

    def apply(self, mod, group):
        if isinstance(mod, nn.Embedding):
            return VocabParallelEmbedding(mod, group, self.sequence_parallel)
        return RowwiseParallelLinear(mod, group, self.sequence_parallel, self.shard_fn, self.input_is_parallel)


@dataclass
class SequenceParallel:
    def apply(self, mod, group):
        return mark_sequence_parallel(mod, group)


def parallelize_module(module: nn.Module, tp_group, plan: dict) -> nn.Module:
    """Replace submodules named in ``plan`` (dotted paths, relative to ``module``) by their TP versions."""
    for name, style in plan.items():
        parent = module
        *path, leaf = name.split(".")
        for p in path:
            parent = getattr(parent, p)
        child = getattr(parent, leaf)
        new = style.apply(child, tp_group)
        if new is not child:
            setattr(parent, leaf, new)
    return module


# ------------------------------------------------------------------------------------------- Llama plan
def parallelize_llama(model, tp_group, sequence_parallel: bool = True, loss_parallel: bool = True,
                      async_tp: int = 0):
    """TP(+SP) plan of fsdp_tp/fsdp_tp_example.py:142-184 for models.llama2.Transformer (fused projections).
    ``async_tp`` = k > 0 (needs sequence_parallel) pipelines each block's sequence all-gathers / reduce-scatters
    against the wqkv / wo / w13 / w2 GEMMs in k micro-collectives (parallel/async_tp.py)."""
    tp = _ws(tp_group)
    args = model.model_args
    hd, nh, nkv = args.head_dim, args.n_heads, args.kv_heads
    assert nh % tp == 0 and nkv % tp == 0, f"heads ({nh}, kv {nkv}) must divide by tp={tp}"
    sp = sequence_parallel
    # token layout of the sequence-parallel activations: async TP deals the tokens in `async_tp` rounds so each of
    # its micro-collectives fills one contiguous slice (comm/functional.py TOKENS)
    cf.set_sp_chunks(tp_group, async_tp if (sp and async_tp) else 1)
    qkv_sizes = [nh * hd, nkv * hd, nkv * hd]
    f = args.ffn_hidden
    assert f % tp == 0, f"ffn hidden {f} must divide by tp={tp}"
    for layer in model.layers:
        a = layer.attention
        a.wqkv = ColwiseParallelLinear(a.wqkv, tp_group, sp, shard_fn=lambda w, g: shard_rows_grouped(w, qkv_sizes, g))
        a.wo = RowwiseParallelLinear(a.wo, tp_group, sp)
        a.n_local_heads, a.n_local_kv_heads = nh // tp, nkv // tp
        ff = layer.feed_forward
        ff.w13 = ColwiseParallelLinear(ff.w13, tp_group, sp, shard_fn=lambda w, g: shard_rows_grouped(w, [f, f], g))
        ff.w2 = RowwiseParallelLinear(ff.w2, tp_group, sp)
        ff.hidden_dim = f // tp
        if sp and async_tp:
            for lin in (a.wqkv, a.wo, ff.w13, ff.w2):
                lin.async_chunks = int(async_tp)
        if sp:
            mark_sequence_parallel(layer.attention_norm, tp_group)
            mark_sequence_parallel(layer.ffn_norm, tp_group)
    model.tok_embeddings = VocabParallelEmbedding(model.tok_embeddings, tp_group, sp)
    if sp:
        mark_sequence_parallel(model.norm, tp_group)
    model.output = ColwiseParallelLinear(model.output, tp_group, sp, gather_output=not loss_parallel)
    model.tp_group = tp_group
    model.sequence_parallel = sp
    model.loss_parallel = loss_parallel
    return model
