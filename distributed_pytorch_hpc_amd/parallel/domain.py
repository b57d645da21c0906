"""Domain (spatial) parallelism: a field too large for one GPU is split along a spatial axis and stencil
operators exchange halos with their neighbours.

The reference only describes this (docs/guide/10_domain_parallel.md:45-149: a single-device halo demo with
torch.cat padding and a pointer to PhysicsNeMo ShardTensor; scripts 07_domain_parallel_* are missing, X1).
Here:
  * ``halo_exchange(x, dim, halo, group)``: pads the local slab with ``halo`` rows from the previous and next
    rank along ``dim`` (zeros at the physical boundary, which is exactly what zero-padded convolution sees);
    backward returns the halo-row gradients to their owners and adds them (exact adjoint).  One
    batch_isend_irecv per exchange; every neighbour pair is a direct xGMI link.
  * ``HaloConv2d``: a stride-1 Conv2d whose padding along the sharded axis is replaced by a halo exchange.
  * ``DomainBatchNorm2d``: batch statistics reduced over the domain group (a field's BN statistics span
    all of its shards), with autograd through the reduction.
  * ``convert_to_domain_parallel(model, group, dim)``: swaps eligible Conv2d / BatchNorm2d in place.
The result is numerically identical to running the unsharded model (tests/test_dist_domain.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from ..comm.functional import all_reduce_sum_partitioned


def _ws(g):
    return dist.get_world_size(g) if dist.is_initialized() else 1


def _rank(g):
    return dist.get_rank(g) if dist.is_initialized() else 0


def _neighbours(group):
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
    r = _rank(group)
    prev = ranks[r - 1] if r > 0 else None
    nxt = ranks[r + 1] if r < len(ranks) - 1 else None
    return prev, nxt


def _exchange(send_lo, send_hi, group, like_lo, like_hi):
    """Send send_lo to prev / send_hi to next; receive from prev into lo, from next into hi."""
    prev, nxt = _neighbours(group)
    recv_lo = torch.zeros_like(like_lo)
    recv_hi = torch.zeros_like(like_hi)
    ops = []
    if prev is not None:
        ops += [dist.P2POp(dist.isend, send_lo.contiguous(), prev, group), dist.P2POp(dist.irecv, recv_lo, prev, group)]
    if nxt is not None:
        ops += [dist.P2POp(dist.isend, send_hi.contiguous(), nxt, group), dist.P2POp(dist.irecv, recv_hi, nxt, group)]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return recv_lo, recv_hi


class _HaloFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, halo, group):
        ctx.dim, ctx.halo, ctx.group = dim, halo, group
        lo = x.narrow(dim, 0, halo)
        hi = x.narrow(dim, x.shape[dim] - halo, halo)
        from_prev, from_next = _exchange(lo, hi, group, lo, hi)
        return torch.cat([from_prev, x, from_next], dim=dim)

    @staticmethod
    def backward(ctx, g):
        dim, halo, group = ctx.dim, ctx.halo, ctx.group
        n = g.shape[dim] - 2 * halo
        g_prev = g.narrow(dim, 0, halo)            # gradient of the rows that belong to prev
        g_next = g.narrow(dim, halo + n, halo)     # ... to next
        core = g.narrow(dim, halo, n).clone()
        back_lo, back_hi = _exchange(g_prev, g_next, group, g_prev, g_next)
        core.narrow(dim, 0, halo).add_(back_lo)
        core.narrow(dim, n - halo, halo).add_(back_hi)
        return core, None, None, None


def halo_exchange(x: torch.Tensor, dim: int, halo: int, group) -> torch.Tensor:
    if halo == 0:
        return x
    if _ws(group) == 1:
        pad = [0, 0] * (x.dim() - dim - 1) + [halo, halo]
        return F.pad(x, pad)
    assert x.shape[dim] >= halo, "local slab thinner than the halo"
    return _HaloFn.apply(x, dim, halo, group)


class HaloConv2d(nn.Module):
    """Conv2d (stride 1 along ``dim``) on an input sharded along ``dim`` (2 = height, 3 = width)."""

    def __init__(self, conv: nn.Conv2d, group, dim: int = 2):
        super().__init__()
        assert conv.stride[dim - 2] == 1 and conv.dilation[dim - 2] == 1, "halo conv needs stride/dilation 1"
        assert isinstance(conv.padding, tuple), "explicit integer padding required"
        self.conv, self.group, self.dim = conv, group, dim
        self.halo = conv.padding[dim - 2]
        self.pad_other = list(conv.padding)
        self.pad_other[dim - 2] = 0

    def forward(self, x):
        x = halo_exchange(x, self.dim, self.halo, self.group)
        c = self.conv
        return F.conv2d(x, c.weight, c.bias, c.stride, tuple(self.pad_other), c.dilation, c.groups)


class DomainBatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d whose training statistics are reduced over the domain group."""

    def __init__(self, bn: nn.BatchNorm2d, group):
        super().__init__(bn.num_features, bn.eps, bn.momentum, bn.affine, bn.track_running_stats)
        self.load_state_dict(bn.state_dict())
        self.group = group
        self.act = getattr(bn, "act", False)   # ops.batchnorm.BatchNormAct2d: act(bn(x) + residual)

    def forward(self, x, residual=None):
        if not self.training:
            y = super().forward(x)
        else:
            y = self._train_forward(x)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if self.act else y

    def _train_forward(self, x):
        n = torch.tensor(float(x.numel() // x.shape[1]), device=x.device)
        s = all_reduce_sum_partitioned(x.sum((0, 2, 3)), self.group)
        ss = all_reduce_sum_partitioned((x * x).sum((0, 2, 3)), self.group)
        cnt = all_reduce_sum_partitioned(n, self.group).detach()
        mean = s / cnt
        var = ss / cnt - mean * mean
        if self.track_running_stats:
            with torch.no_grad():
                m = self.momentum if self.momentum is not None else 0.1
                self.running_mean.mul_(1 - m).add_(mean.detach(), alpha=m)
                self.running_var.mul_(1 - m).add_(var.detach() * cnt / (cnt - 1), alpha=m)
                self.num_batches_tracked += 1
        y = (x - mean[None, :, None, None]) * torch.rsqrt(var + self.eps)[None, :, None, None]
        if self.affine:
            y = y * self.weight[None, :, None, None] + self.bias[None, :, None, None]
        return y


def convert_to_domain_parallel(model: nn.Module, group, dim: int = 2) -> nn.Module:
    """Swap stride-1 Conv2d for HaloConv2d and BatchNorm2d for DomainBatchNorm2d (in place)."""
    for name, child in list(model.named_children()):
        if isinstance(child, nn.Conv2d) and child.stride[dim - 2] == 1 and child.kernel_size[dim - 2] > 1:
            setattr(model, name, HaloConv2d(child, group, dim))
        elif isinstance(child, nn.BatchNorm2d) and not isinstance(child, DomainBatchNorm2d):
            setattr(model, name, DomainBatchNorm2d(child, group))
        else:
            convert_to_domain_parallel(child, group, dim)
    return model
