"""Token embedding (gather + fp32 scatter-add backward, csrc/embedding.hip), vocab-shard aware.

For a vocab-sharded table (TP ``RowwiseParallel`` on tok_embeddings, fsdp_tp/fsdp_tp_example.py:146-149)
ids outside ``[vocab_start, vocab_start + rows)`` produce zero rows locally; the TP layer then
reduce-scatters / all-reduces the partial embeddings.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, table, vocab_start):
        ids = ids.contiguous()
        ctx.save_for_backward(ids)
        ctx.meta = (table.shape[0], vocab_start, table.dtype)
        return _lib.ops().embedding_fwd(ids, table.contiguous(), vocab_start)

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        rows, vstart, dtype = ctx.meta
        dtab = _lib.ops().embedding_bwd(ids, dout.contiguous(), rows, vstart)
        return None, dtab.to(dtype), None


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0) -> torch.Tensor:
    if _lib.use_native(table) and table.shape[1] % 8 == 0 and table.dtype in (torch.bfloat16, torch.float32):
        return _EmbeddingFn.apply(ids, table, vocab_start)
    if vocab_start == 0 and table.shape[0] > 0:
        local = ids
        mask = None
        if ids.numel() and int(ids.max()) >= table.shape[0]:
            mask = ids >= table.shape[0]
            local = ids.masked_fill(mask, 0)
    else:
        local = ids - vocab_start
        mask = (local < 0) | (local >= table.shape[0])
        local = local.masked_fill(mask, 0)
    out = F.embedding(local, table)
    if mask is not None:
        out = out.masked_fill(mask[..., None], 0.0)
    return out


class Embedding(torch.nn.Embedding):
    """nn.Embedding whose GPU path is the CDNA4 gather kernel."""

    def forward(self, ids):
        return embedding(ids, self.weight)
