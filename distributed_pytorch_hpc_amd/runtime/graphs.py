"""Whole training steps as HIP graphs.

The reference has no counterpart (its drivers run eager PyTorch); on MI355X the launch-bound
part of a step -- small models, small per-GPU batches, the dozens of element-wise / norm / optimizer launches
around every GEMM -- costs host time the GPU spends idle.  ``GraphedStep`` records one complete step
(zero-grad, forward, loss, backward, optimizer) into a HIP graph once and replays it: one launch per step, no
Python or autograd bookkeeping on the host.

    step = GraphedStep(lambda x, y: train_step(x, y), warmup=3)
    for x, y in loader:
        loss = step(x, y, lr=sched_lr)      # eager for the first `warmup` calls, then capture + replay

Every call is one real step on its own batch: the first ``warmup`` calls run eagerly on the current stream (lazy
library initialisation, MIOpen / hipBLASLt algorithm selection, allocator warm-up happen outside the capture),
call ``warmup + 1`` captures and then replays, later calls only copy the batch into the graph's static input
buffers and replay.  Requirements, as for any graph: fixed shapes, no host synchronisation inside the step
(``.item()``, data-dependent Python control flow), and an optimizer whose step-dependent scalars live in device
memory -- the engines' fused optimizers switch to that mode (``OptimConfig.capturable``: learning rate and step
count read from a device ``[lr, step]`` tensor by csrc/optim.hip) when a step is graphed; ``torch.optim``
optimizers need ``capturable=True``.  The returned loss is the graph's static output tensor (overwritten by the
next replay): consume or clone it before the next call.

Multi-rank steps would capture their RCCL collectives into the graph too; that path is off unless
``allow_collectives=True`` (not exercised on the 1-GPU test box).

Warm-up runs on the current stream (``warmup_side_stream=True`` warms up on a side stream, the usual capture
recipe).  Round 2 reported replayed ResNet-50 steps diverging with side-stream warm-up; round 3 re-examined
it with ``scripts/diag_graph_side_stream.py`` under MIOpen's deterministic algorithms (two eager runs bitwise equal):
side- and current-stream warm-up, with fresh allocations + writes, in-place writes, or host-synchronised work between
replays, with and without the 1x1 convolution kernels, at 32 px and at 224 px (the 14 x 14 layers) -- every replayed
loss equals the eager one bitwise (``profiles/r3/graph_side_stream_diag_*.json``).  The round-2 comparison ran under
MIOpen's non-deterministic bf16 solvers, where two EAGER runs already differed by a relative update error of 2.1
(``profiles/diag_nondeterminism_resnet*.log``), so its "divergence" had no bitwise baseline; the one blow-up recorded
then (``gpu_tests_intermittent_resnet50_graph_fail.log``) happened with current-stream warm-up, i.e. it was not
tied to the warm-up stream.  ``tests/test_graphs.py::test_graph_warmup_stream_and_interference_bitwise`` keeps both
warm-up modes bitwise-checked against eager with unrelated GPU work between replays.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist


def _engine_of(optimizer):
    return getattr(optimizer, "engine", None)


class GraphedStep:
    """Capture ``step_fn(*tensors) -> loss`` into a HIP graph after ``warmup`` eager calls, then replay it."""

    def __init__(self, step_fn: Callable[..., torch.Tensor], *, optimizer=None, warmup: int = 3,
                 pool=None, allow_collectives: bool = False, warmup_side_stream: bool = False):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU (HIP graphs)")
        if dist.is_initialized() and dist.get_world_size() > 1 and not allow_collectives:
            raise RuntimeError("GraphedStep: multi-rank capture is off (pass allow_collectives=True to record the "
                               "step's RCCL collectives into the graph)")
        self.step_fn = step_fn
        self.warmup = max(int(warmup), 1)
        self.pool = pool
        self.engine = _engine_of(optimizer)
        self.optimizer = optimizer
        if self.engine is not None and self.engine.opt_cfg is not None:
            self.engine.opt_cfg.capturable = True
        elif optimizer is not None and hasattr(optimizer, "param_groups"):
            for g in optimizer.param_groups:
                if "capturable" in g and not g["capturable"]:
                    raise RuntimeError("GraphedStep: construct the torch optimizer with capturable=True")
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_in: list[torch.Tensor] = []
        self.static_out = None
        self._side = torch.cuda.Stream()
        self.warmup_side_stream = warmup_side_stream

    # ---------------------------------------------------------------------------------------------- internals
    def _stage(self, args: Sequence[torch.Tensor]):
        if not self.static_in:
            self.static_in = [a.detach().clone() for a in args]
            return
        if len(args) != len(self.static_in):
            raise ValueError("GraphedStep: number of inputs changed")
        for dst, src in zip(self.static_in, args):
            if src.shape != dst.shape or src.dtype != dst.dtype:
                raise ValueError(f"GraphedStep: input {tuple(src.shape)}/{src.dtype} does not match the captured "
                                 f"{tuple(dst.shape)}/{dst.dtype} (graphs need fixed shapes)")
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)

    def _set_lr(self, lr: Optional[float]):
        if lr is None:
            return
        if self.engine is None and self.optimizer is not None:
            for g in self.optimizer.param_groups:
                if isinstance(g["lr"], torch.Tensor):
                    g["lr"].fill_(lr)
                else:
                    g["lr"] = lr

    def _eager(self, lr):
        if self.engine is not None and lr is not None:
            self.engine.opt_cfg.lr = lr
            if hasattr(self.optimizer, "param_groups"):
                self.optimizer.param_groups[0]["lr"] = lr
        self._set_lr(lr)
        cur = torch.cuda.current_stream()
        side = self._side if self.warmup_side_stream else cur
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            out = self.step_fn(*self.static_in)
        cur.wait_stream(side)
        return out

    def _capture(self):
        # nothing in the capture executes: host-side counters advanced while recording are rolled back, the
        # replays advance them
        saved = self.engine.step_count if self.engine is not None else None
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=self.pool):
            self.static_out = self.step_fn(*self.static_in)
        if self.engine is not None:
            self.engine.step_count = saved

    # ---------------------------------------------------------------------------------------------- public
    def __call__(self, *args: torch.Tensor, lr: Optional[float] = None):
        self._stage(args)
        self.calls += 1
        if self.calls <= self.warmup:
            return self._eager(lr)
        if self.graph is None:
            self._capture()
        if self.engine is not None:
            from ..parallel.data_parallel import graph_replay_prologue

            graph_replay_prologue(self.engine, lr)
            if hasattr(self.optimizer, "param_groups"):
                self.optimizer.param_groups[0]["lr"] = self.engine.opt_cfg.lr
        else:
            self._set_lr(lr)
        self.graph.replay()
        return self.static_out

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def reset(self):
        """Drop the graph (e.g. after a shape change); the next call captures again after no further warm-up."""
        self.graph = None
        self.static_out = None
        self.static_in = []
