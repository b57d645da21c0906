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

import collections
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


# ------------------------------------------------------------------------------------------------ schedules
def chunk_of(k: int, forward: bool, n_stages: int, v: int) -> int:
    """Model chunk run by a rank's k-th forward (or backward) of an interleaved schedule: groups of n_stages
    micro-batches walk the chunks 0..v-1 (backward: v-1..0)."""
    c = (k % (n_stages * v)) // n_stages
    return c if forward else v - 1 - c


def microbatch_of(k: int, n_stages: int, v: int) -> int:
    return (k // (n_stages * v)) * n_stages + k % n_stages


def schedule_plan(n_stages: int, v: int, n_microbatches: int, stage: int) -> list:
    """The op list one pipeline rank executes for a 1F1B step (v = 1) or an interleaved 1F1B step with v model
    chunks per rank (virtual stage of chunk c = c * n_stages + stage; activations move to the next rank, wrapping
    from the last rank's chunk c to rank 0's chunk c + 1).

    Ops: ``("F", k)`` / ``("B", k)`` = the rank's k-th forward / backward (chunk_of / microbatch_of), and
    ``("X", send_fwd, send_bwd, recv_prev_chunk, recv_next_chunk)`` = ONE grouped exchange with the two ring
    neighbours: send the last forward's output to the next rank and / or the last backward's input gradient to the
    previous rank, receive an activation for chunk recv_prev_chunk and / or a gradient for chunk recv_next_chunk
    (None = no receive).  Every rank issues its exchanges in lockstep with its neighbours, so each grouped exchange
    meets the matching group on the peer (deadlock-free under RCCL's per-pair ordering; checked for
    P in 2..8 (v = 1) / 3..8 (v > 1), v in 1..4 by tests/test_dist_pipeline.py).  Warm-up depth: P - s - 1 forwards for v = 1; for v > 1
    2 (P - s - 1) + (v - 1) P (the Megatron-LM interleaved schedule), and everything warm-up when M == P."""
    P, r = n_stages, stage
    total = n_microbatches * v
    if v == 1:
        warm = min(P - r - 1, total)
        all_warm = warm == total
    else:
        if n_microbatches % P:
            raise ValueError(f"interleaved 1F1B needs n_microbatches ({n_microbatches}) divisible by the pipeline "
                             f"size ({P})")
        if P < 3:
            # at P = 2 the ring's next and previous rank coincide: activations and gradients would share one
            # ordered channel per direction and arrive in a different order than the peer receives them
            raise ValueError("interleaved 1F1B needs at least 3 pipeline stages")
        all_warm = n_microbatches == P
        warm = total if all_warm else min(2 * (P - r - 1) + (v - 1) * P, total)
    rem = total - warm

    def first_vs(c):
        return r == 0 and c == 0

    def last_vs(c):
        return r == P - 1 and c == v - 1

    ops = []
    if r != 0:
        ops.append(("X", False, False, 0, None))
    for k in range(warm):
        ops.append(("F", k))
        nc = chunk_of(k + 1, True, P, v)
        recv_prev = not (r == 0 and nc == 0) and k != total - 1
        send_f = not last_vs(chunk_of(k, True, P, v))
        recv_next = k == warm - 1 and not all_warm and r != P - 1
        ops.append(("X", send_f, False, nc if recv_prev else None, v - 1 if recv_next else None))
    for k in range(rem):
        fk = k + warm
        ops.append(("F", fk))
        ops.append(("B", k))
        send_f = not last_vs(chunk_of(fk, True, P, v))
        send_b = not first_vs(chunk_of(k, False, P, v))
        if r == 0:   # what arrives now from the last rank is P - 1 forwards behind (ring wrap to chunk + 1)
            nfc = chunk_of(fk - (P - 1), True, P, v)
            recv_prev = nfc != v - 1
            nfc += 1
        else:
            nfc, recv_prev = chunk_of(fk + 1, True, P, v), True
        if r == P - 1:
            nbc = chunk_of(k - (P - 1), False, P, v)
            recv_next = nbc != 0
            nbc -= 1
        else:
            nbc, recv_next = chunk_of(k + 1, False, P, v), True
        if k == rem - 1:
            recv_prev = False
        ops.append(("X", send_f, send_b, nfc if recv_prev else None, nbc if recv_next else None))
    if all_warm and r != P - 1:
        ops.append(("X", False, False, None, v - 1))
    for k in range(rem, total):
        ops.append(("B", k))
        nbc = chunk_of(k + 1, False, P, v)
        recv_next = not (r == P - 1 and nbc == v - 1) and k != total - 1
        send_b = not first_vs(chunk_of(k, False, P, v))
        ops.append(("X", False, send_b, None, nbc if recv_next else None))
    return [op for op in ops if op[0] != "X" or op[1] or op[2] or op[3] is not None or op[4] is not None]


class _Group:
    """The works of one grouped exchange, waited for at most once (a second wait on a completed gloo receive
    blocks for a message that never comes)."""
    __slots__ = ("works", "keep")

    def __init__(self, works, keep):
        self.works, self.keep = works, keep

    def wait(self):
        for w in self.works:
            w.wait()
        self.works, self.keep = (), ()


class _Received:
    """A tensor whose receive is in flight: the grouped exchange is only waited for when the tensor is consumed
    (RCCL: the compute stream waits on the P2P stream, the host never blocks), so the next micro-batch's compute is
    queued while its neighbours' activations / gradients are still on the xGMI links."""
    __slots__ = ("t", "group")

    def __init__(self, t, group):
        self.t, self.group = t, group

    def get(self):
        self.group.wait()
        return self.t


class PipelineSchedule:
    """Runs one training step of a pipeline stage over ``n_microbatches``.

    ``step(inputs=..., target=...)``: the first stage passes the full-batch input, the last stage the target;
    middle stages pass nothing.  Returns the list of per-micro-batch losses on the last stage (else []).

    schedule: ``"1f1b"`` (default), ``"gpipe"``, or ``"interleaved"`` -- then ``stage_module`` is a list of v model
    chunks (virtual stages c * n_stages + stage, e.g. from ``split_llama_virtual``) and the bubble shrinks to
    (P-1) / (v M + P - 1).  ``dp_engine``: one data-parallel engine over the stage (gradients sync at the rank's
    last backward) or, interleaved, one per chunk (each chunk syncs at its own last backward, so the first chunks'
    reduce-scatter overlaps the remaining backwards).
    """

    def __init__(self, stage_module, stage: int, n_stages: int, n_microbatches: int,
                 loss_fn: Optional[Callable] = None, group=None, schedule: str = "1f1b", device=None,
                 dp_engine=None):
        assert schedule in ("1f1b", "gpipe", "interleaved")
        if isinstance(stage_module, (list, tuple, nn.ModuleList)):
            self.chunks = list(stage_module)
        else:
            self.chunks = [stage_module]
        self.v = len(self.chunks)
        if schedule != "interleaved" and self.v != 1:
            raise ValueError(f"schedule {schedule!r} takes one stage module (got {self.v} chunks)")
        self.module = self.chunks[0] if self.v == 1 else nn.ModuleList(self.chunks)
        self.stage, self.n_stages, self.m = stage, n_stages, n_microbatches
        if schedule == "interleaved":
            schedule_plan(n_stages, self.v, n_microbatches, 0)   # validates M % P == 0 and P >= 3
        self.loss_fn = loss_fn
        self.schedule = schedule
        self.device = device or next(self.chunks[0].parameters()).device
        self.group = group
        self.p2p = P2P(group, stage, n_stages, self.device)
        if group is not None:
            ranks = dist.get_process_group_ranks(group)
        else:
            ranks = list(range(dist.get_world_size())) if dist.is_initialized() else [0]
        self._ring_next = ranks[(stage + 1) % n_stages]
        self._ring_prev = ranks[(stage - 1) % n_stages]
        self.dp_engine = dp_engine
        self.is_first, self.is_last = stage == 0, stage == n_stages - 1
        self._act_meta: Optional[tuple] = None    # (shape, dtype) of every boundary activation / gradient
        self._meta_sent = False

    @property
    def bubble(self) -> float:
        P, M = self.n_stages, self.m
        if self.schedule == "interleaved":
            return (P - 1) / (self.v * M + P - 1)
        return bubble_fraction(P, M)

    # ------------------------------------------------------------------------------------------------
    def _forward(self, x, target_mb, chunk: int = 0):
        y = self.chunks[chunk](x)
        if self.is_last and chunk == self.v - 1:
            loss = self.loss_fn(y, target_mb) if target_mb is not None else y.float().sum()
            return loss, loss
        return y, None

    def _engine_ctx(self, chunk: int, sync: bool):
        eng = self.dp_engine
        if isinstance(eng, (list, tuple)):
            eng = eng[chunk]
        if eng is None or sync:
            return contextlib.nullcontext()
        return eng.no_sync()

    def _backward(self, out, grad, mb_index, chunk: int = 0, sync: Optional[bool] = None):
        if sync is None:
            sync = mb_index == self.m - 1
        with self._engine_ctx(chunk, sync):
            if self.is_last and chunk == self.v - 1:
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
        return self._run_plan(mbs, tgts)

    @torch.no_grad()
    def forward(self, inputs: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Forward-only pipelined pass (evaluation / inference); the last stage returns the concatenated
        outputs of all micro-batches, other stages None.  Interleaved: chunk by chunk, every micro-batch of chunk
        c before chunk c + 1 (the ring order is the same on every rank, so blocking transfers cannot cycle)."""
        mbs = self._split(inputs, "inputs") if self.is_first else [None] * self.m
        self._reset_meta()
        outs, sends = [], []
        for c in range(self.v):
            for i in range(self.m):
                first_vs, last_vs = self.is_first and c == 0, self.is_last and c == self.v - 1
                if first_vs:
                    x = mbs[i]
                elif self.v == 1:
                    x = self.p2p.recv_forward(i == 0)
                else:
                    x = self._recv_blocking(self._ring_prev)
                y = self.chunks[c](x)
                if last_vs:
                    outs.append(y)
                elif self.v == 1:
                    self.p2p.send_forward(y, i == 0)
                else:
                    sends.append(self._send_async(y, self._ring_next))
        for w, _ in sends:
            w.wait()
        return torch.cat(outs, 0) if self.is_last else None

    # ---- transport of the plan executor (ring neighbours, grouped, waits deferred to the consumer) ----
    def _reset_meta(self) -> None:
        # every call (step / forward) re-announces the boundary shape on its first linear-edge send: a later call
        # may run another sequence length or batch size, and receivers must not post buffers of the old shape
        self._act_meta = None
        self._meta_sent = False

    def _needs_header(self) -> bool:
        # only the linear edges stage -> stage + 1 carry the one-time shape header: rank 0 knows the boundary shape
        # from its own first forward before anything arrives over the ring's wrap edge (last rank -> rank 0)
        return not self._meta_sent and self.stage < self.n_stages - 1

    def _send_async(self, y, peer):
        # non-blocking: around the ring every rank sends while its successor may still be sending (a cycle of
        # blocking sends would deadlock); the receives alone order the pass
        if self._needs_header():
            self._send_header(y, peer)
        t = y.detach().contiguous()
        return dist.isend(t, peer, group=self.group), t

    def _recv_blocking(self, peer):
        if self._act_meta is None:
            self._recv_header(peer)
        shape, dtype = self._act_meta
        x = torch.empty(shape, dtype=dtype, device=self.device)
        dist.recv(x, peer, group=self.group)
        return x

    def _send_header(self, y, peer):
        # the first boundary tensor of this call: its shape / dtype, once (all boundaries of one call share them)
        dist.send(self.p2p._header(y), peer, group=self.group)
        self._meta_sent = True
        if self._act_meta is None:
            self._act_meta = (tuple(y.shape), y.dtype)

    def _recv_header(self, peer):
        h = torch.empty(8, dtype=torch.int64, device=self.device)
        dist.recv(h, peer, group=self.group)
        h = h.tolist()
        self._act_meta = (tuple(h[2:2 + h[0]]), _DTYPES[h[1]])

    def _exchange(self, send_f, send_b, recv_prev, recv_next):
        ops, recvd, keep = [], [], []
        if send_f is not None:
            if self._needs_header():
                self._send_header(send_f, self._ring_next)
            elif self._act_meta is None:
                self._act_meta = (tuple(send_f.shape), send_f.dtype)
            t = send_f.detach().contiguous()
            keep.append(t)
            ops.append(dist.P2POp(dist.isend, t, self._ring_next, self.group))
        if send_b is not None:
            t = send_b.contiguous()
            keep.append(t)
            ops.append(dist.P2POp(dist.isend, t, self._ring_prev, self.group))
        if recv_prev:
            if self._act_meta is None:
                self._recv_header(self._ring_prev)
            shape, dtype = self._act_meta
            x = torch.empty(shape, dtype=dtype, device=self.device)
            ops.append(dist.P2POp(dist.irecv, x, self._ring_prev, self.group))
            recvd.append(x)
        if recv_next:
            shape, dtype = self._act_meta
            g = torch.empty(shape, dtype=dtype, device=self.device)
            ops.append(dist.P2POp(dist.irecv, g, self._ring_next, self.group))
            recvd.append(g)
        grp = _Group(dist.batch_isend_irecv(ops) if ops else [], keep)
        return [_Received(t, grp) for t in recvd], grp

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

    def _run_plan(self, mbs, tgts):
        """1F1B / interleaved 1F1B from ``schedule_plan``: forwards, backwards and grouped neighbour exchanges in
        the plan's order; a received tensor is waited for only when its forward / backward starts."""
        P, v, M, r = self.n_stages, self.v, self.m, self.stage
        self._reset_meta()
        fin = [collections.deque() for _ in range(v)]
        gin = [collections.deque() for _ in range(v)]
        saved = [collections.deque() for _ in range(v)]
        per_chunk_engines = isinstance(self.dp_engine, (list, tuple))
        n_bwd = [0] * v
        total_b = 0
        losses, inflight = [], []
        last_out = last_dx = None
        for op in schedule_plan(P, v, M, r):
            if op[0] == "F":
                c, mb = chunk_of(op[1], True, P, v), microbatch_of(op[1], P, v)
                x = mbs[mb] if (r == 0 and c == 0) else self._input(fin[c].popleft().get())
                out, loss = self._forward(x, tgts[mb] if (self.is_last and c == v - 1) else None, c)
                if loss is not None:
                    losses.append(loss.detach())
                saved[c].append((x, out))
                last_out = out
            elif op[0] == "B":
                c, mb = chunk_of(op[1], False, P, v), microbatch_of(op[1], P, v)
                x, out = saved[c].popleft()
                grad = None if (self.is_last and c == v - 1) else gin[c].popleft().get()
                n_bwd[c] += 1
                total_b += 1
                sync = n_bwd[c] == M if per_chunk_engines else total_b == M * v
                self._backward(out, grad, mb, c, sync=sync)
                last_dx = x.grad if not (r == 0 and c == 0) else None
                del x, out
            else:
                _, sf, sb, rp, rn = op
                got, sends = self._exchange(last_out if sf else None, last_dx if sb else None,
                                            rp is not None, rn is not None)
                inflight.append(sends)
                if rp is not None:
                    fin[rp].append(got.pop(0))
                if rn is not None:
                    gin[rn].append(got.pop(0))
                if sf:
                    last_out = None
                if sb:
                    last_dx = None
        for grp in inflight:   # every send has left before its buffers may be reused
            grp.wait()
        assert not any(fin) and not any(gin), "pipeline plan left unconsumed transfers"
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


def partition_by_cost(costs: list, n_parts: int, first_extra: float = 0.0, last_extra: float = 0.0) -> list:
    """Contiguous partition of items with ``costs`` into ``n_parts`` non-empty parts minimising the most expensive
    part, where part 0 also pays ``first_extra`` (embedding) and the last part ``last_extra`` (final norm + LM head +
    loss).  Exact O(n^2 k) dynamic program (n = layers <= a few hundred); ties go to the earliest boundary."""
    n = len(costs)
    if n_parts < 1 or n < n_parts:
        raise ValueError(f"cannot split {n} layers into {n_parts} non-empty stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + float(c))

    def part(i, j, k):   # items [i, j) as part k
        return pre[j] - pre[i] + (first_extra if k == 0 else 0.0) + (last_extra if k == n_parts - 1 else 0.0)

    INF = float("inf")
    best = [[INF] * (n + 1) for _ in range(n_parts + 1)]
    cut = [[0] * (n + 1) for _ in range(n_parts + 1)]
    best[0][0] = 0.0
    for k in range(1, n_parts + 1):
        for j in range(k, n - (n_parts - k) + 1):
            for i in range(k - 1, j):
                if best[k - 1][i] == INF:
                    continue
                val = max(best[k - 1][i], part(i, j, k - 1))
                if val < best[k][j] - 1e-12:
                    best[k][j], cut[k][j] = val, i
    bounds, j = [], n
    for k in range(n_parts, 0, -1):
        i = cut[k][j]
        bounds.append((i, j))
        j = i
    return bounds[::-1]


def llama_costs(model_args, seq_len: int) -> tuple:
    """Modelled training cost (forward + backward FLOPs per token) of each Llama block, of the embedding and of the
    final norm + LM head + cross-entropy: projections x3 (forward + dgrad + wgrad), causal attention forward 1x +
    backward 2.5x (the flash backward recomputes P), memory-bound parts as their FLOP-equivalent at a 2.5 PF / 8 TB/s
    machine balance (~300 FLOP per byte)."""
    a = model_args
    d, kv, hidden = a.dim, a.kv_heads * a.head_dim, a.ffn_hidden
    proj = 2 * (d * d + 2 * d * kv + d * d + 3 * d * hidden)
    attn = 2 * 2 * (seq_len / 2) * d
    block = 3 * proj + 3.5 * attn + 300 * 2 * 12 * d      # + norms / residual / SwiGLU traffic (bf16)
    vocab = a.vocab_size
    head = 3 * 2 * d * vocab + 300 * 2 * 3 * vocab       # LM head GEMMs + logits / CE passes
    emb = 300 * 2 * 3 * d                                # gather forward, scatter-add backward
    return [block] * a.n_layers, emb, head


def _split_bounds(model, n_parts: int, seq_len: Optional[int], costs: Optional[list]) -> list:
    if costs is None and seq_len is None:
        return balanced_split(len(model.layers), n_parts)
    if costs is not None:
        blocks, emb, head = costs
    else:
        blocks, emb, head = llama_costs(model.model_args, seq_len)
    return partition_by_cost(blocks, n_parts, emb, head)


def split_llama(model, n_stages: int, stage: int, seq_len: Optional[int] = None,
                costs: Optional[tuple] = None) -> LlamaStage:
    """Stage ``stage`` of ``n_stages``: equal layer counts by default; with ``seq_len`` (modelled costs,
    ``llama_costs``) or ``costs`` = (per-block costs, embedding, head) the split minimises the most expensive stage,
    counting the embedding on the first and the norm + LM head + loss on the last."""
    lo, hi = _split_bounds(model, n_stages, seq_len, costs)[stage]
    return LlamaStage(model, lo, hi, stage == 0, stage == n_stages - 1)


def split_llama_virtual(model, n_stages: int, v: int, stage: int, seq_len: Optional[int] = None,
                        costs: Optional[tuple] = None) -> nn.ModuleList:
    """The v model chunks rank ``stage`` runs under the interleaved schedule: virtual stages c * n_stages + stage of
    an (n_stages * v)-way split (same balancing options as split_llama)."""
    parts = _split_bounds(model, n_stages * v, seq_len, costs)
    nv = n_stages * v
    return nn.ModuleList([LlamaStage(model, *parts[c * n_stages + stage], c * n_stages + stage == 0,
                                     c * n_stages + stage == nv - 1) for c in range(v)])


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
