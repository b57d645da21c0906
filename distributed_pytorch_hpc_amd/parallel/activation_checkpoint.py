"""Activation checkpointing (recompute-in-backward) with a memory-budget policy sized for 288 GB HBM.

The reference never checkpoints activations.  On MI355X the default is to keep everything (Llama-2-7B with
8 x 4096 tokens per GPU peaks at ~249 GB), so checkpointing is a knob for longer sequences / larger micro-batches:

* ``checkpoint_wrapper(module)`` recomputes ``module``'s forward during backward (non-reentrant
  ``torch.utils.checkpoint``; works with tuple outputs, the fused in-place RoPE, and the data-parallel engines'
  main-grad hooks, which fire during the recomputed backward exactly as without checkpointing);
* ``apply_activation_checkpointing(model, check_fn, every)`` wraps every ``every``-th matching submodule
  (selective checkpointing: ``every=2`` recomputes half of the blocks);
* ``plan_llama_checkpointing(args, batch, seq, hbm_gb)`` estimates the per-block activation bytes of the
  Llama blocks and returns the smallest ``every`` (or 0 = none) that fits a budget.
"""
from __future__ import annotations

from typing import Callable

import torch
from torch import nn
from torch.utils.checkpoint import checkpoint


class CheckpointWrapper(nn.Module):
    """Runs the wrapped module under non-reentrant activation checkpointing while training."""

    def __init__(self, module: nn.Module):
        super().__init__()
        self.module = module

    def forward(self, *args, **kwargs):
        if not (self.training and torch.is_grad_enabled()):
            return self.module(*args, **kwargs)
        return checkpoint(self.module, *args, use_reentrant=False, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._modules["module"], name)


def checkpoint_wrapper(module: nn.Module) -> CheckpointWrapper:
    return CheckpointWrapper(module)


def apply_activation_checkpointing(model: nn.Module, check_fn: Callable[[nn.Module], bool], every: int = 1) -> int:
    """Wrap every ``every``-th submodule for which ``check_fn`` is true (in registration order, in place).

    Returns the number of wrapped modules.  ``every <= 0`` wraps nothing.
    """
    if every <= 0:
        return 0
    count = [0, 0]   # matched, wrapped

    def visit(parent: nn.Module):
        for name, child in list(parent.named_children()):
            if isinstance(child, CheckpointWrapper):
                continue
            if check_fn(child):
                if count[0] % every == 0:
                    setattr(parent, name, CheckpointWrapper(child))
                    count[1] += 1
                count[0] += 1
            else:
                visit(child)

    visit(model)
    return count[1]


def llama_block_activation_bytes(args, batch: int, seq: int, tp: int = 1, dtype_bytes: int = 2) -> int:
    """Saved-for-backward bytes of one models.llama2.TransformerBlock (bf16, flash attention, no dropout).

    Per token: norm outputs (2 x D) + fused QKV (D + 2 kv D) + attention output (D) + residuals (2 x D) +
    W1||W3 output (2 F) + SwiGLU output (F), plus fp32 row statistics; sharded by tp over the hidden dims.
    """
    d, f = args.dim, args.ffn_hidden
    kv = args.kv_heads * args.head_dim
    per_tok = (2 * d + (d + 2 * kv) / tp + d / tp + 2 * d + 3 * f / tp) * dtype_bytes + 16
    return int(per_tok * batch * seq)


def plan_llama_checkpointing(args, batch: int, seq: int, hbm_gb: float = 288.0, static_gb: float = 0.0,
                             reserve_gb: float = 24.0, tp: int = 1) -> int:
    """Smallest checkpoint stride that keeps saved activations within the budget: 0 (none), 1 (every block)…

    ``static_gb``: parameters + gradients + optimizer state already resident on the GPU.
    """
    per_block = llama_block_activation_bytes(args, batch, seq, tp) / 1e9
    budget = hbm_gb - static_gb - reserve_gb
    n = args.n_layers
    if per_block * n <= budget:
        return 0
    # wrapping every k-th block keeps ~n/k block inputs (D per token) instead of their full activations
    inp = 2 * args.dim * batch * seq / 1e9
    for every in (4, 3, 2, 1):
        wrapped = (n + every - 1) // every
        need = (n - wrapped) * per_block + wrapped * inp + per_block   # + one block being recomputed
        if need <= budget:
            return every
    return 1


def apply_llama_checkpointing(model, every: int = 1) -> int:
    from ..models.llama2 import TransformerBlock

    return apply_activation_checkpointing(model, lambda m: isinstance(m, TransformerBlock), every)
