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
