"""Single-node all-reduce over IPC-mapped peer buffers (csrc/custom_allreduce.hip).

The reference leaves every all-reduce to NCCL rings (DDP buckets, C1; Rowwise TP outputs, C11 -- SURVEY.md
§2.12).  On an MI355X node the 8 GPUs are a full xGMI mesh, so a small or medium all-reduce is faster when every
rank reads its peers' buffers directly over all 7 links at once:

* one-shot (<= 256 KiB or 2 ranks): each rank reduces the whole message from all peers -- one barrier;
* two-shot: reduce-scatter by direct peer reads, then all-gather by direct peer reads -- two barriers.

Results are bit-identical on every rank (fp32 accumulation in rank order).  The staging buffers are registered
once (``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle``; handles exchanged with one ``all_gather_object``), so a
call costs one kernel launch and can be captured in a HIP graph.

Use::

    car = XgmiAllReduce(group)            # collective: every rank of the group constructs it
    car.all_reduce(t)                     # in place, SUM (op="avg" divides by the group size)

``get_custom_allreduce(group)`` returns a cached instance, or ``None`` when the group is not eligible (CPU/gloo,
more than 8 ranks, ranks on several hosts, native extension missing).  ``comm.functional.all_reduce_`` routes
eligible messages here when ``DPH_CUSTOM_ALLREDUCE=1`` (off by default; ``benchmarks/comm_bench.py --custom``
measures both paths so the threshold can be set from data on the target node).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib

_ALGOS = {"auto": 0, "oneshot": 1, "twoshot": 2}
_MAX_RANKS = 8


def _group_ranks(group):
    return dist.get_world_size(group), dist.get_rank(group)


class XgmiAllReduce:
    def __init__(self, group=None, max_bytes: int = 64 << 20, timeout_s: float = 10.0, max_blocks: int = 64):
        if not dist.is_initialized():
            raise RuntimeError("XgmiAllReduce needs an initialised process group")
        _lib.require()
        self.group = group
        self.world, self.rank = _group_ranks(group)
        if self.world > _MAX_RANKS:
            raise ValueError(f"XgmiAllReduce supports at most {_MAX_RANKS} ranks (got {self.world})")
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise ValueError("XgmiAllReduce: all ranks of the group must be on one node")
        self.max_bytes = int(max_bytes)
        self.max_blocks = int(max_blocks)
        ops = _lib.ops()
        self._ops = ops
        self.ctx = ops.car_create(self.rank, self.world, self.max_bytes, float(timeout_s))
        mine = ops.car_ipc_handle(self.ctx)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(mine.numpy().tobytes()), group=group)
        table = torch.tensor([list(h) for h in handles], dtype=torch.uint8)
        ops.car_open(self.ctx, table.contiguous())
        dist.barrier(group=group)

    # ------------------------------------------------------------------------------------------------
    def supports(self, t: torch.Tensor) -> bool:
        """Rank-invariant eligibility (shape / dtype / layout only), so every rank takes the same path."""
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and nbytes % 16 == 0 and 0 < nbytes <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor, op: str = "sum", out: Optional[torch.Tensor] = None,
                   algo: str = "auto") -> torch.Tensor:
        """All-reduce ``t`` (in place unless ``out`` is given) and return the result tensor."""
        if not self.supports(t):
            raise ValueError("XgmiAllReduce: tensor must be a contiguous 16-B aligned bf16/fp32 GPU tensor of at most "
                             f"{self.max_bytes} bytes (multiple of 16)")
        if op not in ("sum", "avg"):
            raise ValueError("op must be 'sum' or 'avg'")
        out = t if out is None else out
        scale = 1.0 / self.world if op == "avg" else 1.0
        src = t if t.data_ptr() % 16 == 0 else t.clone()
        dst = out if out.data_ptr() % 16 == 0 else torch.empty_like(out)
        self._ops.car_allreduce(self.ctx, src, dst, _ALGOS[algo], scale, self.max_blocks)
        if dst is not out:
            out.copy_(dst)
        return out

    def errors(self) -> int:
        """Number of barrier timeouts recorded on this rank (0 when healthy)."""
        return int(self._ops.car_status(self.ctx))

    def close(self):
        if getattr(self, "ctx", None):
            self._ops.car_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_CACHE: dict = {}


def custom_allreduce_enabled() -> bool:
    return os.environ.get("DPH_CUSTOM_ALLREDUCE", "0") == "1"


def custom_allreduce_max_bytes() -> int:
    return int(os.environ.get("DPH_CUSTOM_ALLREDUCE_MAX_BYTES", str(8 << 20)))


def get_custom_allreduce(group=None) -> Optional[XgmiAllReduce]:
    """Cached XgmiAllReduce for ``group`` or None if the group cannot use it (collective on first call)."""
    if not dist.is_initialized() or dist.get_backend(group) != "nccl":
        return None
    key = id(group) if group is not None else "world"
    if key not in _CACHE:
        try:
            _CACHE[key] = XgmiAllReduce(group, max_bytes=max(custom_allreduce_max_bytes(), 1 << 20))
        except (ValueError, RuntimeError):
            _CACHE[key] = None
    return _CACHE[key]
