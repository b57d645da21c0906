"""Flat parameter / gradient buffers.

Parameters of a module are re-homed into ONE contiguous buffer per dtype (views, 16-element aligned),
so the optimizer and the gradient collectives each run as a handful of large launches instead of one
per tensor: the fused AdamW kernel sweeps the flat buffer once, DDP all-reduces / FSDP reduce-scatters
contiguous buckets of the flat gradient buffer directly (no pack/unpack copies).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 16  # elements; keeps every view 16-B aligned for bf16 and 64-B aligned for fp32


def align_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class Slot:
    name: str
    offset: int
    numel: int
    shape: torch.Size


class FlatBuffer:
    """A contiguous buffer holding several tensors as aligned views."""

    def __init__(self, shapes: list[tuple[str, torch.Size]], dtype: torch.dtype, device, pad_to: int = 1,
                 fill: float | None = 0.0):
        self.slots: list[Slot] = []
        off = 0
        for name, shape in shapes:
            n = int(torch.Size(shape).numel())
            self.slots.append(Slot(name, off, n, torch.Size(shape)))
            off = align_up(off + n)
        self.numel = align_up(max(off, 1), max(pad_to, 1))
        self.dtype = dtype
        self.device = torch.device(device)
        self.data = torch.empty(self.numel, dtype=dtype, device=self.device)
        if fill is not None:
            self.data.fill_(fill)

    def view(self, i: int) -> torch.Tensor:
        s = self.slots[i]
        return self.data[s.offset: s.offset + s.numel].view(s.shape)

    def views(self) -> list[torch.Tensor]:
        return [self.view(i) for i in range(len(self.slots))]


def flatten_params_(params: list[torch.nn.Parameter], pad_to: int = 1) -> FlatBuffer:
    """Move the storage of ``params`` (same dtype/device) into one FlatBuffer; params become views."""
    assert params, "no parameters"
    dtype, device = params[0].dtype, params[0].device
    for p in params:
        assert p.dtype == dtype and p.device == device, "flatten_params_: mixed dtype/device"
    fb = FlatBuffer([(str(i), p.shape) for i, p in enumerate(params)], dtype, device, pad_to=pad_to, fill=0.0)
    with torch.no_grad():
        for i, p in enumerate(params):
            v = fb.view(i)
            v.copy_(p.data)
            p.data = v
    return fb


def _cl4(t: torch.Tensor) -> bool:
    """4-D tensor stored channels-last (and not also plain-contiguous, e.g. a 1x1 kernel)."""
    return t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last)


def flat_order(t: torch.Tensor) -> torch.Tensor:
    """``t`` flattened in its storage order: NHWC for channels-last 4-D tensors, row-major otherwise."""
    return t.permute(0, 2, 3, 1).reshape(-1) if _cl4(t) else t.reshape(-1)


def flat_order_like(value: torch.Tensor, like: torch.Tensor, name: str | None = None) -> torch.Tensor:
    """A logically-shaped ``value`` (any strides, e.g. from a state dict) flattened in ``like``'s storage order, i.e.
    the element order ``like`` has inside an engine's flat buffer (inverse of ``param_view(...).contiguous()``).
    The shapes must match exactly: a same-numel tensor of another shape (e.g. a transposed weight) would otherwise
    load silently in scrambled order."""
    if tuple(value.shape) != tuple(like.shape):
        raise ValueError(f"size mismatch for {name or 'parameter'}: copying a param with shape {tuple(value.shape)}, "
                         f"the shape in the current model is {tuple(like.shape)}")
    return value.permute(0, 2, 3, 1).reshape(-1) if _cl4(like) else value.reshape(-1)


def param_view(flat_slice: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """View of a flat-buffer slice shaped like ``like``, channels-last when ``like`` is, so a channels-last
    convolution weight living in an engine's flat bucket is read in place by MIOpen instead of being copied to NHWC
    on every call.  Pairs with ``flat_order`` (same element order).  The flat layout (hence sharded optimizer state)
    follows the model's memory format: resume with the format it was saved with."""
    if _cl4(like):
        n, c, h, w = like.shape
        return flat_slice.view(n, h, w, c).permute(0, 3, 1, 2)
    return flat_slice.view(like.shape)
