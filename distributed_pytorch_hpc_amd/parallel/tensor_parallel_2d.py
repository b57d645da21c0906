"""2-D tensor parallelism on a (rows x cols) process grid (doc-only in the reference:
docs/guide/06_tensor_parallel.md:105-128, "2D TP splits along both dimensions using a 2D GPU grid ... See the
scripts for a working example" -- no script exists).

Layout (grid coordinates (i, j), ``row`` group = ranks sharing i, ``col`` group = ranks sharing j):
  * activations X [..., T, K]: rank (i, j) holds the block X[T_i, K_j] -- tokens split over grid rows, features
    over grid columns.  Every Linear2D maps this layout to the same layout of its output, so layers chain with
    no redistribution in between.
  * Linear2D(K -> N) weight W [N, K]: rank (i, j) holds W[N_j, K_i] (output features over columns, input features
    over rows): N*K / (rows*cols) parameters per rank, nothing replicated.

Forward (two all-gathers, no all-reduce):
    X[T_i, :]  = all_gather over the row group of X[T_i, K_j]        (along K)
    W[N_j, :]  = all_gather over the col group of W[N_j, K_i]        (along K)
    Y[T_i, N_j] = X[T_i, :] @ W[N_j, :]^T                            (local GEMM)
Backward = the adjoints: dX is reduce-scattered over the row group, dW over the col group (comm/functional.py
gather_along_dim pairs).  Per-rank traffic is O(T K / rows + N K / cols) instead of 1-D TP's all-reduce of
[T, N] over all P ranks: on a 2 x 4 grid of one MI355X node every message crosses 1 xGMI hop and is split over
~sqrt(P) peers.  Row-wise statistics (RMSNorm / LayerNorm over the feature dim) reduce over the row group.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn

from ..comm import functional as cf
from ..comm.mesh import Mesh
from .linear import linear as _linear


class Grid2D(Mesh):
    """(rows, cols) mesh; ``row_group`` = ranks with the same row index, ``col_group`` = same column index."""

    def __init__(self, rows: int, cols: int, backend: str | None = None):
        super().__init__((rows, cols), ("i", "j"), backend)
        self.rows, self.cols = rows, cols
        self.i, self.j = self.coords
        # the group that varies j (same i) is the mesh dim "j"
        self.row_group, self.col_group = self.groups["j"], self.groups["i"]


def _chunk(x: torch.Tensor, n: int, k: int, dim: int) -> torch.Tensor:
    assert x.shape[dim] % n == 0, f"dim {dim} ({x.shape[dim]}) not divisible by {n}"
    return x.chunk(n, dim)[k].contiguous()


def shard_activation_2d(x: torch.Tensor, grid: Grid2D, token_dim: int = -2) -> torch.Tensor:
    """Full activation [..., T, K] -> this rank's block [..., T/rows, K/cols]."""
    return _chunk(_chunk(x, grid.rows, grid.i, token_dim), grid.cols, grid.j, -1)


def gather_activation_2d(x: torch.Tensor, grid: Grid2D, token_dim: int = -2) -> torch.Tensor:
    """Inverse of shard_activation_2d (no autograd; for checks and outputs)."""
    x = cf.all_gather_dim(x, x.dim() - 1, grid.row_group)
    return cf.all_gather_dim(x, token_dim % x.dim(), grid.col_group)


class Linear2D(nn.Module):
    """2-D tensor-parallel replacement for ``nn.Linear`` (see module docstring)."""

    def __init__(self, lin: nn.Linear, grid: Grid2D):
        super().__init__()
        self.grid = grid
        w = lin.weight.detach()
        self.in_features, self.out_features = lin.in_features, lin.out_features
        self.weight = nn.Parameter(_chunk(_chunk(w, grid.cols, grid.j, 0), grid.rows, grid.i, 1),
                                   requires_grad=lin.weight.requires_grad)
        self.bias = None
        if lin.bias is not None:
            # b[N_j] replicated down a grid column: its gradient sums the column's token blocks
            self.bias = nn.Parameter(_chunk(lin.bias.detach(), grid.cols, grid.j, 0))
            if grid.rows > 1:
                self.bias.register_hook(lambda g, grp=grid.col_group: cf.all_reduce_(g.contiguous().clone(), grp))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xg = cf.gather_along_dim(x, x.dim() - 1, self.grid.row_group)       # [.., T_i, K]
        wg = cf.gather_along_dim(self.weight, 1, self.grid.col_group)       # [N_j, K]
        return _linear(xg, wg, self.bias)

    def extra_repr(self):
        return (f"in={self.in_features}, out={self.out_features}, grid={self.grid.rows}x{self.grid.cols}, "
                f"local_weight={tuple(self.weight.shape)}")


class RMSNorm2D(nn.Module):
    """RMSNorm over a feature dim that is split across the row group (weight sharded like the features)."""

    def __init__(self, norm: nn.Module, grid: Grid2D):
        super().__init__()
        self.grid = grid
        self.eps = norm.eps
        self.dim = norm.weight.numel()
        self.weight = nn.Parameter(_chunk(norm.weight.detach(), grid.cols, grid.j, 0))
        if grid.rows > 1:
            self.weight.register_hook(lambda g, grp=grid.col_group: cf.all_reduce_(g.contiguous().clone(), grp))

    def forward(self, x):
        xf = x.float()
        ss = cf.all_reduce_sum_partitioned(xf.pow(2).sum(-1, keepdim=True), self.grid.row_group)
        return (xf * torch.rsqrt(ss / self.dim + self.eps)).type_as(x) * self.weight


class LayerNorm2D(nn.Module):
    """LayerNorm over a feature dim split across the row group."""

    def __init__(self, norm: nn.LayerNorm, grid: Grid2D):
        super().__init__()
        self.grid = grid
        self.eps = norm.eps
        self.dim = norm.normalized_shape[-1]
        self.weight = nn.Parameter(_chunk(norm.weight.detach(), grid.cols, grid.j, 0))
        self.bias = nn.Parameter(_chunk(norm.bias.detach(), grid.cols, grid.j, 0)) if norm.bias is not None else None
        if grid.rows > 1:
            for p in (self.weight, self.bias):
                if p is not None:
                    p.register_hook(lambda g, grp=grid.col_group: cf.all_reduce_(g.contiguous().clone(), grp))

    def forward(self, x):
        xf = x.float()
        s = cf.all_reduce_sum_partitioned(torch.cat([xf.sum(-1, keepdim=True), xf.pow(2).sum(-1, keepdim=True)], -1),
                                          self.grid.row_group)
        mean = s[..., :1] / self.dim
        var = (s[..., 1:] / self.dim - mean * mean).clamp_min(0)
        y = ((xf - mean) * torch.rsqrt(var + self.eps)).type_as(x) * self.weight
        return y + self.bias if self.bias is not None else y


def parallelize_2d(module: nn.Module, grid: Grid2D) -> nn.Module:
    """Replace every nn.Linear / nn.LayerNorm / RMSNorm-like module (``weight`` + ``eps``) in ``module`` by its 2-D
    version.  Element-wise modules need no change (they act on local blocks)."""
    for name, child in list(module.named_children()):
        if isinstance(child, nn.Linear):
            setattr(module, name, Linear2D(child, grid))
        elif isinstance(child, nn.LayerNorm):
            setattr(module, name, LayerNorm2D(child, grid))
        elif hasattr(child, "weight") and hasattr(child, "eps") and not list(child.children()) \
                and isinstance(getattr(child, "weight"), torch.Tensor) and child.weight.dim() == 1:
            setattr(module, name, RMSNorm2D(child, grid))
        else:
            parallelize_2d(child, grid)
    return module


def mse_loss_2d(pred: torch.Tensor, target: torch.Tensor, grid: Grid2D) -> tuple[torch.Tensor, torch.Tensor]:
    """Mean squared error of 2-D-sharded blocks.  Returns (local loss to backprop -- the blocks' share of the
    global mean, so the sum over ranks is the global loss -- and the global loss value for logging)."""
    n = pred.numel() * grid.rows * grid.cols
    local = (pred.float() - target.float()).pow(2).sum() / n
    tot = local.detach().clone()
    if dist.is_initialized() and grid.rows * grid.cols > 1:
        dist.all_reduce(tot)
    return local, tot
