"""Fused optimizers over flat buffers (csrc/optim.hip).

``FusedAdamW`` / ``FusedSGD`` are drop-in ``torch.optim.Optimizer`` subclasses with the exact update
rules of torch.optim.AdamW / SGD (the reference drivers use AdamW(foreach=True) -- e.g.
fsdp_tp/fsdp_tp_example.py:194 -- and SGD(momentum=0.9) -- scripts/main.py:309-311).  At construction
the parameters of each group are re-homed into one flat buffer per (dtype, device), gradients are
pre-allocated views of a matching flat buffer, and every ``step()`` is ONE kernel launch per buffer.

bf16 parameters get an fp32 master copy inside the optimizer (mixed-precision training); fp32
parameters are updated in place.  An optional device scalar ``grad_scale`` (see ``clip_grad_norm_``)
multiplies gradients inside the kernel, so gradient clipping needs no host synchronisation.
"""
from __future__ import annotations

import math
from collections import defaultdict

import torch

from ..ops import _lib
from ..utils.flat import FlatBuffer, flatten_params_


class _FlatState:
    def __init__(self, params: list[torch.nn.Parameter], momentum_buffers: int):
        self.params = params
        self.pbuf = flatten_params_(params)
        self.gbuf = FlatBuffer([(str(i), p.shape) for i, p in enumerate(params)], self.pbuf.dtype,
                               self.pbuf.device, fill=0.0)
        for i, p in enumerate(params):
            p.grad = self.gbuf.view(i)
        if self.pbuf.dtype == torch.float32:
            self.master = self.pbuf.data
            self.param_out = None
        else:
            self.master = self.pbuf.data.float()
            self.param_out = self.pbuf.data
        self.bufs = [torch.zeros_like(self.master) for _ in range(momentum_buffers)]
        self.step = 0

    def gather_grads(self):
        """Make sure every param.grad lives in the flat gradient buffer (zero_grad(set_to_none) safe)."""
        for i, p in enumerate(self.params):
            slot = self.gbuf.view(i)
            g = p.grad
            if g is None:
                slot.zero_()
            elif g.data_ptr() != slot.data_ptr():
                slot.copy_(g)
            p.grad = slot

    def zero_grad(self):
        self.gbuf.data.zero_()
        for i, p in enumerate(self.params):
            p.grad = self.gbuf.view(i)


def _group_flat(params, momentum_buffers):
    by_key = defaultdict(list)
    for p in params:
        if p.requires_grad:
            by_key[(p.dtype, p.device)].append(p)
    return [_FlatState(ps, momentum_buffers) for ps in by_key.values()]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._flat = [_group_flat(g["params"], 2) for g in self.param_groups]
        self.grad_scale: torch.Tensor | None = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group, flats in zip(self.param_groups, self._flat):
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            for fs in flats:
                fs.gather_grads()
                fs.step += 1
                bc1 = 1.0 - b1 ** fs.step
                bc2 = 1.0 - b2 ** fs.step
                m, v = fs.bufs
                g = fs.gbuf.data
                if _lib.use_native(fs.master):
                    _lib.ops().adamw_step_(fs.master, m, v, g, fs.param_out, lr, b1, b2, eps, wd, bc1, bc2,
                                           self.grad_scale)
                else:
                    adamw_reference_(fs.master, m, v, g, lr, b1, b2, eps, wd, bc1, bc2, self.grad_scale)
                    if fs.param_out is not None:
                        fs.param_out.copy_(fs.master)
        return loss

    def zero_grad(self, set_to_none: bool = False):
        for flats in self._flat:
            for fs in flats:
                fs.zero_grad()

    def flat_states(self):
        return [fs for flats in self._flat for fs in flats]

    # state_dict: per-flat master/m/v + step (rank-local; the ckpt module shards/consolidates it)
    def state_dict(self):
        out = {"param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
               "flat": []}
        for fs in self.flat_states():
            out["flat"].append({"step": fs.step, "master": fs.master.detach().cpu(),
                                "exp_avg": fs.bufs[0].cpu(), "exp_avg_sq": fs.bufs[1].cpu()})
        return out

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        for fs, st in zip(self.flat_states(), sd["flat"]):
            fs.step = int(st["step"])
            fs.master.copy_(st["master"])
            fs.bufs[0].copy_(st["exp_avg"])
            fs.bufs[1].copy_(st["exp_avg_sq"])
            if fs.param_out is not None:
                fs.param_out.copy_(fs.master)


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        self._flat = [_group_flat(g["params"], 1) for g in self.param_groups]
        self.grad_scale: torch.Tensor | None = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group, flats in zip(self.param_groups, self._flat):
            for fs in flats:
                fs.gather_grads()
                first = fs.step == 0
                fs.step += 1
                g = fs.gbuf.data
                if _lib.use_native(fs.master):
                    _lib.ops().sgd_step_(fs.master, fs.bufs[0], g, fs.param_out, group["lr"], group["momentum"],
                                         group["dampening"], group["weight_decay"], group["nesterov"], first,
                                         self.grad_scale)
                else:
                    sgd_reference_(fs.master, fs.bufs[0], g, group["lr"], group["momentum"], group["dampening"],
                                   group["weight_decay"], group["nesterov"], first, self.grad_scale)
                    if fs.param_out is not None:
                        fs.param_out.copy_(fs.master)
        return loss

    def zero_grad(self, set_to_none: bool = False):
        for flats in self._flat:
            for fs in flats:
                fs.zero_grad()

    def flat_states(self):
        return [fs for flats in self._flat for fs in flats]

    def state_dict(self):
        return {"param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
                "flat": [{"step": fs.step, "master": fs.master.cpu(), "momentum_buffer": fs.bufs[0].cpu()}
                         for fs in self.flat_states()]}

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        for fs, st in zip(self.flat_states(), sd["flat"]):
            fs.step = int(st["step"])
            fs.master.copy_(st["master"])
            fs.bufs[0].copy_(st["momentum_buffer"])
            if fs.param_out is not None:
                fs.param_out.copy_(fs.master)


# ------------------------------------------------------------------------------------------ references
def _skip(grad_scale) -> bool:
    """A NaN gradient scale skips the update, as in the HIP kernels (csrc/optim.hip: the xGMI health guard)."""
    return torch.is_tensor(grad_scale) and bool(torch.isnan(grad_scale).any())


def adamw_reference_(master, m, v, g, lr, b1, b2, eps, wd, bc1, bc2, grad_scale=None):
    if _skip(grad_scale):
        return
    gf = g.float()
    if grad_scale is not None:
        gf = gf * grad_scale
    master.mul_(1.0 - lr * wd)
    m.lerp_(gf, 1.0 - b1)
    v.mul_(b2).addcmul_(gf, gf, value=1.0 - b2)
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)


def sgd_reference_(master, buf, g, lr, momentum, dampening, wd, nesterov, first, grad_scale=None):
    if _skip(grad_scale):
        return
    d = g.float()
    if grad_scale is not None:
        d = d * grad_scale
    if wd:
        d = d + wd * master
    if momentum:
        if first:
            buf.copy_(d)
        else:
            buf.mul_(momentum).add_(d, alpha=1.0 - dampening)
        d = d + momentum * buf if nesterov else buf
    master.add_(d, alpha=-lr)


def global_grad_norm(tensors: list[torch.Tensor]) -> torch.Tensor:
    """sqrt(sum of squares) over flat gradient tensors, as a device scalar (no host sync)."""
    dev = tensors[0].device
    acc = torch.zeros(1, dtype=torch.float32, device=dev)
    for t in tensors:
        if _lib.use_native(t) and t.is_contiguous():
            _lib.ops().sumsq_(t, acc)
        else:
            acc += t.float().pow(2).sum()
    return acc.sqrt()


def clip_grad_norm_(optimizer, max_norm: float, extra_sumsq: torch.Tensor | None = None) -> torch.Tensor:
    """Global-norm clipping folded into the next optimizer kernel via ``optimizer.grad_scale``.

    ``extra_sumsq`` lets a sharded engine add the all-reduced sum of squares of other ranks' shards.
    Returns the (device) total norm.
    """
    flats = optimizer.flat_states()
    for fs in flats:
        fs.gather_grads()
    sq = global_grad_norm([fs.gbuf.data for fs in flats]) ** 2
    if extra_sumsq is not None:
        sq = sq + extra_sumsq
    norm = sq.sqrt()
    optimizer.grad_scale = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    return norm
