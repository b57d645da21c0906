"""Pipeline parallelism: stage split, P2P activation/gradient transport, GPipe and 1F1B schedules.

Capability parity with scripts/04_pipeline_parallel_pp/ (manual send/recv split 01_manual_model_split.py:53-153,
torch.distributed.pipelining GPipe/1F1B in 02_pipeline_schedules.py and 03_pipeline_training.py:123-296), with
the reference defects fixed:
  * the loss function always sees flattened [mb*S, V] logits vs [mb*S] targets for LM stages;
  * the bubble is reported as the idle FRACTION (S-1)/(M+S-1), the same for GPipe and 1F1B (1F1B's gain is the
    peak number of in-flight activations: S - s instead of M);
  * forward AND backward are pipelined (the manual reference is forward-only);
  * PP x DP: a stage can be wrapped by the data-parallel engine over its dp group; gradient collectives are
    deferred to the last micro-batch's backward (engine.no_sync for the others).

Transport is one RCCL send/recv per micro-batch per boundary (every GPU pair is a direct xGMI link on an
MI355X node); opposite-direction transfers of the steady 1F1B phase are posted together with
``batch_isend_irecv`` so neighbouring stages never deadlock on blocking sends.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch import nn

_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32]


def bubble_fraction(n_stages: int, n_microbatches: int) -> float:
    """Idle fraction of a GPipe/1F1B step: (S-1) / (M+S-1)."""
    return (n_stages - 1) / (n_microbatches + n_stages - 1)


class P2P:
    """Neighbour transport inside a pipeline group (ranks given as GLOBAL ranks)."""

    def __init__(self, group, stage: int, n_stages: int, device):
        self.group = group
        self.stage, self.n_stages = stage, n_stages
        if group is not None:
            ranks = dist.get_process_group_ranks(group)
        else:
            ranks = list(range(dist.get_world_size())) if dist.is_initialized() else [0]
        self.prev = ranks[stage - 1] if stage > 0 else None
        self.next = ranks[stage + 1] if stage < n_stages - 1 else None
        self.device = device
        self.fwd_meta: Optional[tuple] = None   # (shape, dtype) of activations received from prev

    def _header(self, t: torch.Tensor) -> torch.Tensor:
        h = torch.zeros(8, dtype=torch.int64, device=self.device)
        h[0] = t.dim()
        h[1] = _DTYPES.index(t.dtype)
        for i, s in enumerate(t.shape):
            h[2 + i] = s
        return h

    def send_forward(self, y: torch.Tensor, with_header: bool):
        if self.next is None:
            return
        if with_header:
            dist.send(self._header(y), self.next, group=self.group)
        dist.send(y.detach().contiguous(), self.next, group=self.group)

    def recv_forward(self, with_header: bool) -> torch.Tensor:
        if with_header or self.fwd_meta is None:
            h = torch.empty(8, dtype=torch.int64, device=self.device)
            dist.recv(h, self.prev, group=self.group)
            h = h.tolist()
            self.fwd_meta = (tuple(h[2:2 + h[0]]), _DTYPES[h[1]])
        shape, dtype = self.fwd_meta
        x = torch.empty(shape, dtype=dtype, device=self.device)
        dist.recv(x, self.prev, group=self.group)
        return x

    def send_backward(self, dx: torch.Tensor):
        if self.prev is None or dx is None:
            return
        dist.send(dx.contiguous(), self.prev, group=self.group)

    def recv_backward(self, like: torch.Tensor) -> torch.Tensor:
        g = torch.empty_like(like)
        dist.recv(g, self.next, group=self.group)
        return g

    def send_forward_recv_backward(self, y: torch.Tensor) -> torch.Tensor:
        g = torch.empty_like(y)
        ops = [dist.P2POp(dist.isend, y.detach().contiguous(), self.next, self.group),
               dist.P2POp(dist.irecv, g, self.next, self.group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return g

    def send_backward_recv_forward(self, dx: Optional[torch.Tensor]) -> torch.Tensor:
        shape, dtype = self.fwd_meta
        x = torch.empty(shape, dtype=dtype, device=self.device)
        ops = [dist.P2POp(dist.irecv, x, self.prev, self.group)]
        if dx is not None:
            ops.insert(0, dist.P2POp(dist.isend, dx.contiguous(), self.prev, self.group))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return x


class PipelineSchedule:
    """Runs one training step of a pipeline stage over ``n_microbatches``.

    ``step(inputs=..., target=...)``: the first stage passes the full-batch input, the last stage the target;
    middle stages pass nothing.  Returns the list of per-micro-batch losses on the last stage (else []).
    """

    def __init__(self, stage_module: nn.Module, stage: int, n_stages: int, n_microbatches: int,
                 loss_fn: Optional[Callable] = None, group=None, schedule: str = "1f1b", device=None,
                 dp_engine=None):
        assert schedule in ("1f1b", "gpipe")
        self.module = stage_module
        self.stage, self.n_stages, self.m = stage, n_stages, n_microbatches
        self.loss_fn = loss_fn
        self.schedule = schedule
        self.device = device or next(stage_module.parameters()).device
        self.p2p = P2P(group, stage, n_stages, self.device)
        self.dp_engine = dp_engine
        self.is_first, self.is_last = stage == 0, stage == n_stages - 1

    @property
    def bubble(self) -> float:
        return bubble_fraction(self.n_stages, self.m)

    # ------------------------------------------------------------------------------------------------
    def _forward(self, x, target_mb):
        y = self.module(x)
        if self.is_last:
            loss = self.loss_fn(y, target_mb) if target_mb is not None else y.float().sum()
            return loss, loss
        return y, None

    def _backward(self, out, grad, mb_index):
        ctx = contextlib.nullcontext()
        if self.dp_engine is not None and mb_index != self.m - 1:
            ctx = self.dp_engine.no_sync()
        with ctx:
            if self.is_last:
                (out / self.m).backward()
            else:
                out.backward(grad)

    def _input(self, x):
        if x.is_floating_point():
            x.requires_grad_(True)
        return x

    def _split(self, t: torch.Tensor, what: str) -> list:
        # every micro-batch must have micro-batch 0's shape: only that one carries a shape header (P2P.recv_forward)
        if t.shape[0] % self.m:
            raise ValueError(f"pipeline {what}: batch {t.shape[0]} is not divisible by n_microbatches={self.m}")
        return list(t.chunk(self.m, 0))

    def step(self, inputs: Optional[torch.Tensor] = None, target: Optional[torch.Tensor] = None) -> list:
        mbs = self._split(inputs, "inputs") if self.is_first else [None] * self.m
        tgts = self._split(target, "target") if (self.is_last and target is not None) else [None] * self.m
        if self.schedule == "gpipe":
            return self._gpipe(mbs, tgts)
        return self._1f1b(mbs, tgts)

    @torch.no_grad()
    def forward(self, inputs: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Forward-only pipelined pass (evaluation / inference); the last stage returns the concatenated
        outputs of all micro-batches, other stages None."""
        mbs = self._split(inputs, "inputs") if self.is_first else [None] * self.m
        outs = []
        for i in range(self.m):
            x = mbs[i] if self.is_first else self.p2p.recv_forward(i == 0)
            y = self.module(x)
            if self.is_last:
                outs.append(y)
            else:
                self.p2p.send_forward(y, i == 0)
        return torch.cat(outs, 0) if self.is_last else None

    def _recv_fwd(self, mbs, i, with_header):
        return mbs[i] if self.is_first else self._input(self.p2p.recv_forward(with_header))

    def _gpipe(self, mbs, tgts):
        saved, losses = [], []
        for i in range(self.m):
            x = self._recv_fwd(mbs, i, i == 0)
            out, loss = self._forward(x, tgts[i])
            if loss is not None:
                losses.append(loss.detach())
            self.p2p.send_forward(out, i == 0) if not self.is_last else None
            saved.append((x, out))
        for i in range(self.m):
            x, out = saved[i]
            grad = None if self.is_last else self.p2p.recv_backward(out)
            self._backward(out, grad, i)
            if not self.is_first:
                self.p2p.send_backward(x.grad)
        return losses

    def _1f1b(self, mbs, tgts):
        warmup = min(self.n_stages - self.stage - 1, self.m)
        remaining = self.m - warmup
        saved, losses = [], []
        fwd_i = bwd_i = 0
        for _ in range(warmup):
            x = self._recv_fwd(mbs, fwd_i, fwd_i == 0)
            out, loss = self._forward(x, tgts[fwd_i])
            if loss is not None:
                losses.append(loss.detach())
            if not self.is_last:
                self.p2p.send_forward(out, fwd_i == 0)
            saved.append((x, out))
            fwd_i += 1
        x = self._recv_fwd(mbs, fwd_i, fwd_i == 0) if remaining > 0 else None
        for j in range(remaining):
            out, loss = self._forward(x, tgts[fwd_i])
            if loss is not None:
                losses.append(loss.detach())
            saved.append((x, out))
            first_send = fwd_i == 0
            fwd_i += 1
            if self.is_last:
                grad = None
            elif first_send:  # only when warmup == 0 on a non-last stage (cannot happen for M >= 1)
                self.p2p.send_forward(out, True)
                grad = self.p2p.recv_backward(out)
            else:
                grad = self.p2p.send_forward_recv_backward(out)
            bx, bout = saved[bwd_i]
            self._backward(bout, grad, bwd_i)
            saved[bwd_i] = None
            bwd_i += 1
            dx = bx.grad if not self.is_first else None
            if j == remaining - 1:
                if not self.is_first:
                    self.p2p.send_backward(dx)
            else:
                if self.is_first:
                    x = mbs[fwd_i]
                else:
                    x = self._input(self.p2p.send_backward_recv_forward(dx))
        for _ in range(warmup):
            bx, bout = saved[bwd_i]
            grad = None if self.is_last else self.p2p.recv_backward(bout)
            self._backward(bout, grad, bwd_i)
            saved[bwd_i] = None
            bwd_i += 1
            if not self.is_first:
                self.p2p.send_backward(bx.grad)
        return losses


# ------------------------------------------------------------------------------------------------ splitting
def balanced_split(n_items: int, n_stages: int) -> list[tuple[int, int]]:
    base, rem = divmod(n_items, n_stages)
    out, s = [], 0
    for i in range(n_stages):
        e = s + base + (1 if i < rem else 0)
        out.append((s, e))
        s = e
    return out


class LlamaStage(nn.Module):
    """A contiguous slice of a models.llama2.Transformer: [embedding] + layers[lo:hi] + [norm + output + loss]."""

    def __init__(self, model, lo: int, hi: int, first: bool, last: bool):
        super().__init__()
        self.first, self.last = first, last
        self.tok_embeddings = model.tok_embeddings if first else None
        self.layers = nn.ModuleList(list(model.layers)[lo:hi])
        self.norm = model.norm if last else None
        self.output = model.output if last else None
        self.model_args = model.model_args

    def forward(self, x):
        h = self.tok_embeddings(x) if self.first else x
        delta = None
        for layer in self.layers:
            h, delta = layer(h, delta)
        if self.last:
            if delta is None:
                y = self.norm(h)
            else:
                _, y = self.norm(h, delta)
            return self.output(y)
        return h if delta is None else h + delta


def split_llama(model, n_stages: int, stage: int) -> LlamaStage:
    lo, hi = balanced_split(len(model.layers), n_stages)[stage]
    return LlamaStage(model, lo, hi, stage == 0, stage == n_stages - 1)


def split_sequential(seq: nn.Sequential, n_stages: int, stage: int) -> nn.Sequential:
    lo, hi = balanced_split(len(seq), n_stages)[stage]
    return nn.Sequential(*list(seq)[lo:hi])


def lm_loss(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Cross-entropy with the [B, S, V] -> [B*S, V] flattening the reference's PP driver missed (X3)."""
    from .. import ops

    return ops.fused_cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), inplace=False)


def make_lm_loss(tp_group=None, loss_parallel: bool = False) -> Callable:
    """Last-stage loss for Llama pipelines; with TP loss-parallel the stage emits vocab-sharded logits
    [mb, S, V/tp] and the loss is the vocab-parallel cross-entropy (no [mb, S, V] all-gather)."""
    if not (loss_parallel and tp_group is not None):
        return lm_loss
    from .. import ops

    def loss(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        vloc = logits.shape[-1]
        return ops.vocab_parallel_cross_entropy(logits.reshape(-1, vloc), target.reshape(-1),
                                                dist.get_rank(tp_group) * vloc, tp_group)

    return loss
