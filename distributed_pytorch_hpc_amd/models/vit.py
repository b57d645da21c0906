"""SimpleViT for gridded weather regression (capability parity with
scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:82-202; 6,906,176 parameters at the reference config).

Same modules and parameter names (patch_embed.proj, pos_embed, blocks[i].{norm1, attn.{q,k,v,out}_proj, norm2,
mlp.{fc1, fc2}}, norm, head) so the reference TP plan (q/k/v/fc1 column-parallel, out_proj/fc2 row-parallel)
applies unchanged.  On the GPU: LayerNorm and GELU run the CDNA4 kernels and attention is the non-causal
flash kernel instead of the reference's materialised softmax(QK^T) (no [B, h, N, N] scores in HBM).
Head counts are taken from the (possibly TP-sharded) projection width, as the reference's reshape(B, N, -1, hd).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops


class PatchEmbed(nn.Module):
    """Non-overlapping k = s = p patch projection (tensor_parallel_vit.py:82-90) computed as ONE GEMM: patches are
    disjoint, so the "convolution" is a reshape of the image into [B, N_patches, C*p*p] rows times the flattened
    [E, C*p*p] kernel -- no im2col, no implicit-GEMM convolution search.  The parameter stays a
    Conv2d weight so state dicts match the reference."""

    def __init__(self, in_channels: int, embed_dim: int, patch_size: int):
        super().__init__()
        self.patch = patch_size
        self.proj = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        b, c, h, w = x.shape
        p = self.patch
        hp, wp = h // p, w // p
        if h != hp * p or w != wp * p:   # Conv2d drops the remainder rows / columns
            x = x[:, :, :hp * p, :wp * p]
        rows = x.reshape(b, c, hp, p, wp, p).permute(0, 2, 4, 1, 3, 5).reshape(b, hp * wp, c * p * p)
        wt = self.proj.weight.reshape(self.proj.out_channels, c * p * p)
        return F.linear(rows, wt, self.proj.bias)


class Attention(nn.Module):
    def __init__(self, dim: int, num_heads: int):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.q_proj = nn.Linear(dim, dim)
        self.k_proj = nn.Linear(dim, dim)
        self.v_proj = nn.Linear(dim, dim)
        self.out_proj = nn.Linear(dim, dim)

    def forward(self, x):
        b, n, _ = x.shape
        q = self.q_proj(x).reshape(b, n, -1, self.head_dim)
        k = self.k_proj(x).reshape(b, n, -1, self.head_dim)
        v = self.v_proj(x).reshape(b, n, -1, self.head_dim)
        o = ops.flash_attention(q, k, v, causal=False, scale=self.scale)
        return self.out_proj(o.reshape(b, n, -1))


class MLP(nn.Module):
    def __init__(self, dim: int, hidden_dim: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden_dim)
        self.act = ops.GELU()
        self.fc2 = nn.Linear(hidden_dim, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class TransformerBlock(nn.Module):
    def __init__(self, dim: int, num_heads: int, mlp_ratio: int = 4):
        super().__init__()
        self.norm1 = ops.LayerNorm(dim)
        self.attn = Attention(dim, num_heads)
        self.norm2 = ops.LayerNorm(dim)
        self.mlp = MLP(dim, int(dim * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class SimpleViT(nn.Module):
    def __init__(self, in_channels: int = 65, out_channels: int = 65, patch_size: int = 8, lat: int = 64,
                 lon: int = 128, embed_dim: int = 256, depth: int = 6, num_heads: int = 8, mlp_ratio: int = 4):
        super().__init__()
        self.patch_size, self.out_channels = patch_size, out_channels
        self.h_patches, self.w_patches = lat // patch_size, lon // patch_size
        self.patch_embed = PatchEmbed(in_channels, embed_dim, patch_size)
        self.pos_embed = nn.Parameter(torch.randn(1, self.h_patches * self.w_patches, embed_dim) * 0.02)
        self.blocks = nn.ModuleList([TransformerBlock(embed_dim, num_heads, mlp_ratio) for _ in range(depth)])
        self.norm = ops.LayerNorm(embed_dim)
        self.head = nn.Linear(embed_dim, out_channels * patch_size * patch_size)

    def forward(self, x):
        b = x.shape[0]
        x = self.patch_embed(x) + self.pos_embed
        for blk in self.blocks:
            x = blk(x)
        x = self.head(self.norm(x))
        p = self.patch_size
        x = x.reshape(b, self.h_patches, self.w_patches, self.out_channels, p, p)
        return x.permute(0, 3, 1, 4, 2, 5).reshape(b, self.out_channels, self.h_patches * p, self.w_patches * p)


def vit_tp_plan(sequence_parallel: bool = False) -> dict:
    """The reference ViT TP plan (tensor_parallel_vit.py:352-361) for parallel.parallelize_module."""
    from ..parallel.tensor_parallel import ColwiseParallel, RowwiseParallel

    plan = {}
    for i in range(6):
        for n in ("q_proj", "k_proj", "v_proj"):
            plan[f"blocks.{i}.attn.{n}"] = ColwiseParallel()
        plan[f"blocks.{i}.attn.out_proj"] = RowwiseParallel()
        plan[f"blocks.{i}.mlp.fc1"] = ColwiseParallel()
        plan[f"blocks.{i}.mlp.fc2"] = RowwiseParallel()
    return plan
