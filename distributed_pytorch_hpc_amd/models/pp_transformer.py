"""PipelineTransformer (capability parity with scripts/04_pipeline_parallel_pp/03_pipeline_training.py:51-120;
11,700,736 parameters at vocab 10000 / dim 256 / 8 heads / 4 stages x 2 layers).

Token + learned positional embedding, four named stages (``stage0..stage3``) of pre-LN encoder blocks, final
LayerNorm and a bias-free vocabulary projection.  The multi-head attention keeps nn.MultiheadAttention's packed
parameters (``in_proj_weight/in_proj_bias``, ``out_proj``) but runs the CDNA4 flash kernel (non-causal, like the
reference), attention dropout included (in-kernel counter-hash mask, ops/attention.py).  ``stage_modules()``
yields the per-stage callables for parallel.pipeline.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops


class PackedMHA(nn.Module):
    def __init__(self, dim: int, n_heads: int, dropout: float = 0.0):
        super().__init__()
        self.n_heads, self.head_dim, self.dropout = n_heads, dim // n_heads, dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * dim, dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * dim))
        self.out_proj = nn.Linear(dim, dim)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, x):
        b, s, d = x.shape
        qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias).view(b, s, 3, -1, self.head_dim)
        q, k, v = qkv.unbind(2)
        o = ops.flash_attention(q, k, v, causal=False, dropout_p=self.dropout if self.training else 0.0)
        return self.out_proj(o.reshape(b, s, d))


class EncoderBlock(nn.Module):
    def __init__(self, dim: int, n_heads: int, dropout: float = 0.1):
        super().__init__()
        self.norm1 = ops.LayerNorm(dim)
        self.attn = PackedMHA(dim, n_heads, dropout)
        self.norm2 = ops.LayerNorm(dim)
        self.ffn = nn.Sequential(nn.Linear(dim, 4 * dim), ops.GELU(), nn.Linear(4 * dim, dim), nn.Dropout(dropout))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.ffn(self.norm2(x))


class Embed(nn.Module):
    def __init__(self, vocab_size: int, dim: int, max_pos: int = 1024):
        super().__init__()
        self.embedding = ops.Embedding(vocab_size, dim)
        self.pos_encoding = ops.Embedding(max_pos, dim)

    def forward(self, tokens):
        pos = torch.arange(tokens.shape[1], device=tokens.device).unsqueeze(0)
        return self.embedding(tokens) + self.pos_encoding(pos)


class Head(nn.Module):
    def __init__(self, dim: int, vocab_size: int):
        super().__init__()
        self.norm = ops.LayerNorm(dim)
        self.output = nn.Linear(dim, vocab_size, bias=False)

    def forward(self, x):
        return self.output(self.norm(x))


class PipelineTransformer(nn.Module):
    def __init__(self, vocab_size: int = 10000, dim: int = 256, n_heads: int = 8, layers_per_stage: int = 2,
                 n_stages: int = 4, dropout: float = 0.1):
        super().__init__()
        self.n_stages = n_stages
        self.embed = Embed(vocab_size, dim)
        for i in range(n_stages):
            setattr(self, f"stage{i}", nn.Sequential(*[EncoderBlock(dim, n_heads, dropout)
                                                       for _ in range(layers_per_stage)]))
        self.head = Head(dim, vocab_size)

    def forward(self, tokens):
        x = self.embed(tokens)
        for i in range(self.n_stages):
            x = getattr(self, f"stage{i}")(x)
        return self.head(x)

    def stage_modules(self, n_pipeline_stages: int | None = None) -> list[nn.Module]:
        """Stage i of an n-stage pipeline: [embed] + stage blocks + [head]."""
        n = n_pipeline_stages or self.n_stages
        assert self.n_stages % n == 0
        per = self.n_stages // n
        out = []
        for s in range(n):
            mods = [getattr(self, f"stage{s * per + j}") for j in range(per)]
            if s == 0:
                mods.insert(0, self.embed)
            if s == n - 1:
                mods.append(self.head)
            out.append(nn.Sequential(*mods))
        return out
