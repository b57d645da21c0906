"""Losses: fused softmax cross-entropy (csrc/xent.hip) and the latitude-weighted MSE of the ERA5
drivers (scripts/01_data_parallel_ddp/multinode_ddp_unet.py:221-229).

``fused_cross_entropy`` computes the mean loss AND writes d(loss)/d(logits) in place over the logits
during the forward kernel; backward only scales that buffer by the incoming scalar gradient.  This
removes the reference's fp32 [B, S, V] logits copy (llama2_model.py:447) and a separate softmax pass.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib


class _FusedXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing):
        valid = (target != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / valid).reshape(1)
        need_grad = ctx.needs_input_grad[0]
        loss_rows, _ = _lib.ops().cross_entropy_fwd(logits, target, inv, ignore_index, need_grad, smoothing)
        if need_grad:
            # the kernel overwrote the logits buffer with d(loss)/d(logits) (a raw in-place write that the
            # autograd version counter does not see; nothing else saved these logits for backward)
            ctx.grad_buf = logits
        return loss_rows.sum() * inv[0]

    @staticmethod
    def backward(ctx, gloss):
        g = ctx.grad_buf
        ctx.grad_buf = None
        g.mul_(gloss.to(g.dtype))
        return g, None, None, None


def fused_cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                        label_smoothing: float = 0.0, inplace: bool = True) -> torch.Tensor:
    """Mean cross-entropy over rows of [N, V] logits.  With ``inplace`` (default) the logits buffer is
    consumed (overwritten by its gradient) -- pass ``inplace=False`` if the caller still needs it."""
    if logits.dim() != 2:
        logits = logits.reshape(-1, logits.shape[-1])
        target = target.reshape(-1)
    if _lib.use_native(logits) and logits.dtype in (torch.bfloat16, torch.float32):
        if not inplace:
            logits = logits.clone()
        return _FusedXentFn.apply(logits, target.contiguous(), ignore_index, float(label_smoothing))
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, label_smoothing=label_smoothing)


_LAT_W: dict = {}


def latitude_weights(n_lat: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """cos(latitude) weights over a [90, -90] grid normalised to mean 1 (multinode_ddp_unet.py:221-229).
    Cached per (n_lat, device, dtype): built once on the host, so a HIP-graph capture of the loss finds them
    resident (a host-to-device copy is not allowed while a stream is capturing)."""
    key = (int(n_lat), str(torch.device(device) if device is not None else "cpu"), dtype)
    w = _LAT_W.get(key)
    if w is None:
        lat = torch.linspace(90.0, -90.0, n_lat, dtype=torch.float64)
        w = torch.cos(lat * math.pi / 180.0)
        w = (w / w.mean()).to(device=device, dtype=dtype)
        _LAT_W[key] = w
    return w


class _LatMseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, n_global, lat_offset):
        ctx.save_for_backward(pred, target)
        ctx.n_global, ctx.lat_offset = n_global, lat_offset
        return _lib.ops().latmse_fwd(pred, target, n_global, lat_offset)

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        need_t = ctx.needs_input_grad[1]
        dp, dt = _lib.ops().latmse_bwd(g.float().reshape(1), pred, target, ctx.n_global, ctx.lat_offset, need_t)
        return dp, (dt if need_t else None), None, None


def latitude_weighted_mse(pred: torch.Tensor, target: torch.Tensor, n_lat_global: int | None = None,
                          lat_offset: int = 0) -> torch.Tensor:
    """mean over [B, C, H, W] of w[H] * (pred - target)^2.

    For a latitude-sharded field (domain parallelism) pass the global latitude count and this shard's first
    row: the weights are the matching slice of the global cos-latitude profile, so the average of the
    per-shard losses over equal shards is the global loss.  GPU tensors run csrc/latmse.hip (weights computed
    in-kernel from the row index, one reduction pass, deterministic); CPU tensors the PyTorch expression."""
    n = n_lat_global or pred.shape[-2]
    if (pred.dim() == 4 and _lib.use_native(pred) and pred.dtype in (torch.bfloat16, torch.float32)
            and target.dtype == pred.dtype and target.shape == pred.shape):
        # channels-last when either operand is laid out channel-innermost (a channels-last tensor, or a strided
        # channels-last view such as the first Cout columns of a padded 1x1 convolution's output): one compaction
        # copy at most, never an NHWC <-> NCHW transpose of both fields
        cl = (pred.is_contiguous(memory_format=torch.channels_last) and not pred.is_contiguous()) or (
            pred.stride(1) == 1 and pred.shape[1] > 1 and target.is_contiguous(memory_format=torch.channels_last))
        fmt = torch.channels_last if cl else torch.contiguous_format
        p, t = pred.contiguous(memory_format=fmt), target.contiguous(memory_format=fmt)
        p = p if p.data_ptr() % 16 == 0 else p.clone(memory_format=fmt)
        t = t if t.data_ptr() % 16 == 0 else t.clone(memory_format=fmt)
        return _LatMseFn.apply(p, t, int(n), int(lat_offset))
    w = latitude_weights(n, pred.device, torch.float32)[lat_offset:lat_offset + pred.shape[-2]].view(1, 1, -1, 1)
    return (w * (pred.float() - target.float()).pow(2)).mean()


def vocab_parallel_cross_entropy(local_logits: torch.Tensor, target: torch.Tensor, vocab_start: int, group,
                                 ignore_index: int = -100) -> torch.Tensor:
    """Cross-entropy over vocab-sharded logits [N, V/tp] without gathering the vocab dim ("loss
    parallel"): two [N] all-reduces (max, sum-exp) and one [N] all-reduce of the target logit."""
    from ..comm.functional import all_reduce_autograd_max, all_reduce_autograd_sum

    x = local_logits.float()
    n, vloc = x.shape
    m = all_reduce_autograd_max(x.detach().max(dim=-1).values, group)
    e = torch.exp(x - m[:, None])
    se = all_reduce_autograd_sum(e.sum(-1), group)
    local_t = target - vocab_start
    in_range = (local_t >= 0) & (local_t < vloc)
    idx = local_t.clamp(0, vloc - 1)
    tl = x.gather(1, idx[:, None]).squeeze(1) * in_range
    tl = all_reduce_autograd_sum(tl, group)
    loss = torch.log(se) + m - tl
    valid = target != ignore_index
    return (loss * valid).sum() / valid.sum().clamp_min(1)
