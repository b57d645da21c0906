"""Data-parallel engine: flat bucketed gradients, RCCL collectives overlapped with backward, fused (optionally
sharded) optimizer.  Backs both ``DDP`` (all-reduce, replicated optimizer state) and ``FSDP``
(reduce-scatter + sharded fp32 master/optimizer state + parameter all-gather, i.e. ZeRO-2 semantics with
parameters resident -- the right trade on a 288 GB MI355X -- plus ZeRO-3 units, see fsdp.py).

Reference capability: DDP(model, device_ids=[local_rank]) (scripts/01_data_parallel_ddp/*, scripts/main.py:258)
and FSDP(model, auto_wrap_policy, ShardingStrategy, MixedPrecision) (scripts/02_fully_sharded_fsdp/
resnet_fsdp_training.py:193-212).  The design here is MI355X-first rather than a wrapper of torch's DDP/FSDP:

  * All trainable parameters live in ONE flat buffer (param dtype) laid out in reverse registration order
    (~ backward production order) and cut into buckets at parameter boundaries.  Gradients live in a flat
    buffer with the same layout; ``Linear`` weights receive dW from the backward GEMM directly
    (parallel/linear.py), other parameters via a post-accumulate-grad hook.  No pack/unpack copies.
  * A bucket's collective is launched (async, RCCL's own stream waits on the compute stream) as soon as it
    and every earlier bucket are complete -- a fixed launch order on every rank -- and overlaps the
    remaining backward.  Bucket size defaults to 256 MiB: on the 7-link xGMI mesh RCCL all-reduce /
    reduce-scatter reach their plateau bus bandwidth well below that, and a 7B model still gets ~50
    buckets to pipeline against the backward pass (benchmarks/comm_bench.py measures the curve).
  * The optimizer (fused AdamW / SGD kernels, csrc/optim.hip) runs per bucket on the rank's shard:
    wait(reduce-scatter_b) -> adamw(shard_b) -> all-gather_b (async), buckets taken in forward order.  The next
    forward only waits for the all-gather of the bucket a module actually needs (forward pre-hook), so parameter
    all-gathers overlap the next step's forward.
  * 1/world averaging and optional global-norm clipping are folded into the optimizer kernel through a
    device scalar: no extra pass, no host sync.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from functools import partial
from typing import Optional

import torch
import torch.distributed as dist
from torch import nn

from ..comm import custom_allreduce as _car
from ..comm.custom_allreduce import check_health as check_xgmi_health
from ..comm.custom_allreduce import use_custom as use_custom_allreduce
from ..ops import _lib
from ..train import optim as optim_ref
from ..utils.flat import ALIGN, align_up, param_view
from .linear import convert_linears_, join_wgrad_stream, wgrad_stream


@dataclass
class MixedPrecision:
    """torch.distributed.fsdp.MixedPrecision-compatible policy (resnet_fsdp_training.py:198-204)."""
    param_dtype: Optional[torch.dtype] = None
    reduce_dtype: Optional[torch.dtype] = None
    buffer_dtype: Optional[torch.dtype] = None


@dataclass
class OptimConfig:
    name: str = "adamw"
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 1e-2
    momentum: float = 0.0
    dampening: float = 0.0
    nesterov: bool = False
    max_grad_norm: Optional[float] = None
    # read lr / step from device memory (HIP-graph capturable step; runtime/graphs.py turns it on)
    capturable: bool = False


class StepHyper:
    """Device-resident ``[lr, step]`` read by the fused optimizer kernels in capturable mode (csrc/optim.hip
    ``hyper``): a HIP graph captured around ``engine.step()`` then replays the right learning rate and bias
    corrections every step.  Eagerly the host writes both values (two tiny fills, no sync); inside a capture
    only the device-side ``step += 1`` is recorded, and the host sets the learning rate before each replay."""

    def __init__(self, device):
        self.t = torch.zeros(2, dtype=torch.float32, device=device)

    def advance(self, lr: float, step: int):
        if self.t.is_cuda and torch.cuda.is_current_stream_capturing():
            self.t[1:2].add_(1.0)
        else:
            self.t[0:1].fill_(lr)
            self.t[1:2].fill_(float(step))

    def set_lr(self, lr: float):
        self.t[0:1].fill_(lr)


def _hyper_for(engine, native: bool):
    """The engine's StepHyper tensor (advanced for this step) when its optimizer is capturable and native."""
    cfg = engine.opt_cfg
    if not (cfg.capturable and native):
        return None
    if engine._hyper is None:
        engine._hyper = StepHyper(engine.device)
    engine._hyper.advance(cfg.lr, engine.step_count)
    return engine._hyper.t


def graph_replay_prologue(engine, lr: Optional[float] = None):
    """Host side of one replayed step: the learning rate goes to device memory, the host step count follows."""
    if lr is not None:
        engine.opt_cfg.lr = lr
    if engine._hyper is not None:
        engine._hyper.set_lr(engine.opt_cfg.lr)
    engine.step_count += 1


class _Bucket:
    __slots__ = ("idx", "params", "offset", "numel", "shard_numel", "shard_offset", "n_ready", "launched",
                 "work", "ag_work", "opt_event")

    def __init__(self, idx):
        self.idx = idx
        self.params: list[nn.Parameter] = []
        self.offset = 0
        self.numel = 0
        self.shard_numel = 0
        self.shard_offset = 0
        self.n_ready = 0
        self.launched = False
        self.work = None
        self.ag_work = None
        self.opt_event = None


class DataParallelEngine:
    def __init__(self, module: nn.Module, process_group=None, shard: bool = False,
                 mixed_precision: Optional[MixedPrecision] = None, bucket_cap_mb: float = 256.0,
                 overlap: bool = True, convert_linears: bool = True, broadcast_from_rank0: bool = True,
                 overlap_step: Optional[bool] = None):
        self.module = module
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.shard = shard and self.world > 1
        self.overlap = overlap
        mp = mixed_precision or MixedPrecision()
        if mp.param_dtype is not None:
            for p in module.parameters():
                p.data = p.data.to(mp.param_dtype)
        if mp.buffer_dtype is not None:
            for b in module.buffers():
                if b.is_floating_point():
                    b.data = b.data.to(mp.buffer_dtype)
        if convert_linears:
            convert_linears_(module)

        seen, params = set(), []
        for p in module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        assert params, "no trainable parameters"
        self.params = params
        self.param_dtype = params[0].dtype
        self.device = params[0].device
        for p in params:
            assert p.dtype == self.param_dtype, "DataParallelEngine: all parameters must share one dtype"
        self.grad_dtype = mp.reduce_dtype or self.param_dtype
        self.is_gloo = dist.is_initialized() and dist.get_backend(process_group) == "gloo"

        # ---- bucket assignment (reverse registration order ~ gradient production order) ----
        if bucket_cap_mb == "auto":   # alpha-beta fit of the collective (comm/cost_model.py, $DPH_COMM_FIT)
            from ..comm.cost_model import auto_bucket_mb

            grad_bytes = sum(p.numel() for p in params) * torch.empty((), dtype=self.grad_dtype).element_size()
            bucket_cap_mb = auto_bucket_mb(grad_bytes, self.world, self.shard)
        self.bucket_cap_mb = float(bucket_cap_mb)
        cap = max(int(bucket_cap_mb * 2 ** 20 / params[0].element_size()), 1)
        pad = ALIGN * self.world
        buckets, cur, cur_n = [], _Bucket(0), 0
        for p in reversed(params):
            n = align_up(p.numel())
            if cur.params and cur_n + n > cap:
                buckets.append(cur)
                cur, cur_n = _Bucket(len(buckets)), 0
            cur.params.append(p)
            cur_n += n
        if cur.params:
            buckets.append(cur)
        off = soff = 0
        for b in buckets:
            b.offset = off
            b.numel = align_up(sum(align_up(p.numel()) for p in b.params), pad)
            b.shard_numel = b.numel // self.world
            b.shard_offset = soff
            off += b.numel
            soff += b.shard_numel
        self.buckets = buckets
        self.total = off
        self.shard_total = soff

        # ---- flat buffers; parameters and main grads become views ----
        self.flat_param = torch.zeros(self.total, dtype=self.param_dtype, device=self.device)
        self.flat_grad = torch.zeros(self.total, dtype=self.grad_dtype, device=self.device)
        self._bucket_of = {}
        with torch.no_grad():
            for b in buckets:
                o = b.offset
                for p in b.params:
                    n = p.numel()
                    v = param_view(self.flat_param[o:o + n], p)   # channels-last weights stay channels-last
                    v.copy_(p.data)
                    p.main_grad = param_view(self.flat_grad[o:o + n], p)
                    p._dph_persistent_grad = True   # flat_grad lives as long as the engine (ops.conv.zero_bias_grad)
                    p._dph_zeroed = False
                    p.data = v
                    p._dph_accum = False
                    p._dph_grad_ready = partial(self._on_grad_ready, p)
                    self._bucket_of[id(p)] = b
                    p._dph_flat_off = o
                    o += align_up(n)
        self._hooks = [p.register_post_accumulate_grad_hook(self._post_accumulate) for p in params]
        if broadcast_from_rank0 and self.world > 1:
            dist.broadcast(self.flat_param, src=dist.get_global_rank(process_group, 0) if process_group else 0,
                           group=process_group)

        # ---- optimizer-side buffers (fp32 master, sharded when self.shard) ----
        n_opt = self.shard_total if self.shard else self.total
        self.master = torch.empty(n_opt, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for b in buckets:
                self.master_view(b).copy_(self.param_shard_view(b))
        self.grad_shard = (torch.zeros(self.shard_total, dtype=self.grad_dtype, device=self.device)
                           if self.shard else None)
        self.opt_state: list[torch.Tensor] = []
        self.opt_cfg: Optional[OptimConfig] = None
        self.step_count = 0
        self._hyper: Optional[StepHyper] = None
        self._sync_enabled = True
        self._tp_due = False
        self._next_launch = 0
        self._callback_queued = False
        self._gscale = torch.full((1,), 1.0 / self.world, dtype=torch.float32, device=self.device)
        self._init_tp_partial()

        # Opt-in (overlap_step=True / DPH_OVERLAP_STEP=1): each bucket's update runs on a side stream in forward
        # order and the next forward waits per module for its bucket only, so the HBM-bound AdamW / SGD sweep can
        # overlap the MFMA-bound forward GEMMs.  Bit-identical results (tests/test_engine.py), but measured +0.1 % on
        # the Llama-2-7B bench (27,896 vs 27,867 tok/s, interleaved A/B on one MI355X, profiles/ab/overlap_step_*):
        # the library GEMMs hold every CU, so the side-stream sweep mostly runs between them, not beside them.
        if overlap_step is None:
            overlap_step = os.environ.get("DPH_OVERLAP_STEP", "0") == "1"
        self.overlap_step = bool(overlap_step) and self.device.type == "cuda"
        self._opt_stream = None

        # forward pre-hooks: wait for the all-gather (sharded) / the optimizer update (overlapped step) of the
        # buckets holding a module's own parameters; the root's post-hook joins the optimizer stream completely
        self._fwd_hooks = []
        for m in module.modules():
            ids = {self._bucket_of[id(p)].idx for p in m.parameters(recurse=False) if id(p) in self._bucket_of}
            if ids:
                self._fwd_hooks.append(m.register_forward_pre_hook(partial(self._wait_ag, sorted(ids))))
        self._fwd_hooks.append(module.register_forward_hook(lambda *_: self._join_opt_stream()))

    # ------------------------------------------------------------------------------------------ TP-partial grads
    def _init_tp_partial(self):
        """Sequence-parallel parameters (norm weights that run on a sequence shard, tensor_parallel.py
        mark_sequence_parallel) hold gradients that are partial over the TP group.  Instead of one latency-bound
        all-reduce per parameter from a backward hook (65 per Llama-2-7B backward), the engine takes them over: the
        data-parallel reduction runs as usual (a sum, so the order of the two reductions does not matter) and
        ``step`` completes them with ONE all-reduce over the TP group of every such element this rank holds (the
        flat / sharded layouts are identical across TP ranks: equal shard shapes).  SURVEY.md C9."""
        groups = {}
        for p in self.params:
            g = getattr(p, "_dph_sp_group", None)
            if getattr(p, "_dph_sequence_parallel", False) and g is not None and dist.is_initialized() and \
                    dist.get_world_size(g) > 1:
                groups.setdefault(id(g), (g, []))[1].append(p)
        self._tp_partial = []
        for g, ps in groups.values():
            idx = []
            for p in ps:
                p._dph_tp_batched = True
                b, o, n = self._bucket_of[id(p)], p._dph_flat_off, p.numel()
                if not self.shard:
                    idx.append(torch.arange(o, o + n, dtype=torch.int64))
                    continue
                lo = b.offset + self.rank * b.shard_numel           # this rank's shard of the bucket
                s0, s1 = max(o, lo), min(o + n, lo + b.shard_numel)
                if s0 < s1:
                    idx.append(torch.arange(s0 - lo, s1 - lo, dtype=torch.int64) + b.shard_offset)
            cat = torch.cat(idx) if idx else torch.zeros(0, dtype=torch.int64)
            self._tp_partial.append((g, cat.to(self.device)))

    def finish_grad_sync(self):
        """The one place gradient synchronisation completes: wait for every bucket's data-parallel reduction, then
        (once per reduction round) finish the sequence-parallel gradients over the TP group.  ``synchronize`` and
        ``step`` both call it, so ``main_grad`` read after ``synchronize()`` -- grad-norm logging, gradient checks,
        external optimizers -- is already complete over TP."""
        for b in self.buckets:
            self._wait_reduce(b)
        # only after a reduction round has launched: synchronize() inside no_sync(), or before the first backward,
        # must not all-reduce partial SP sums that later micro-steps still add to (they would be counted tp times)
        if self._tp_partial and self._tp_due:
            self._reduce_tp_partial()
            self._tp_due = False
        check_xgmi_health()

    def _reduce_tp_partial(self):
        from ..comm.functional import all_reduce_

        red = self.grad_shard if self.shard else self.flat_grad
        for g, idx in self._tp_partial:
            # every rank of the TP group joins the collective, even one whose shard holds none of the elements; the
            # message is small, so below the measured crossover it takes the direct-peer path (all_reduce_)
            buf = red.index_select(0, idx) if idx.numel() else torch.zeros(8, dtype=red.dtype, device=red.device)
            all_reduce_(buf, g)
            if idx.numel():
                red.index_copy_(0, idx, buf)

    # ------------------------------------------------------------------------------------------ views
    def grad_view(self, b: _Bucket) -> torch.Tensor:
        return self.flat_grad[b.offset:b.offset + b.numel]

    def param_view(self, b: _Bucket) -> torch.Tensor:
        return self.flat_param[b.offset:b.offset + b.numel]

    def param_shard_view(self, b: _Bucket) -> torch.Tensor:
        if self.shard:
            s = b.offset + self.rank * b.shard_numel
            return self.flat_param[s:s + b.shard_numel]
        return self.param_view(b)

    def grad_shard_view(self, b: _Bucket) -> torch.Tensor:
        if self.shard:
            return self.grad_shard[b.shard_offset:b.shard_offset + b.shard_numel]
        return self.grad_view(b)

    def master_view(self, b: _Bucket) -> torch.Tensor:
        if self.shard:
            return self.master[b.shard_offset:b.shard_offset + b.shard_numel]
        return self.master[b.offset:b.offset + b.numel]

    # ------------------------------------------------------------------------------------------ grads
    def _post_accumulate(self, p: torch.Tensor):
        g = p.grad
        if g is None:
            return
        mg = p.main_grad
        p._dph_zeroed = False
        with torch.no_grad():
            if p._dph_accum:
                mg.add_(g)
            else:
                mg.copy_(g)
                p._dph_accum = True
        p.grad = None
        self._on_grad_ready(p)

    def _on_grad_ready(self, p):
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
        b = self._bucket_of[id(p)]
        if b.launched:
            raise RuntimeError("DataParallelEngine: a parameter produced a gradient after its bucket was "
                               "reduced (parameter used twice in one backward?); construct with overlap=False")
        b.n_ready += 1
        if self.overlap and self._sync_enabled:
            self._launch_ready()

    def _launch_ready(self):
        while self._next_launch < len(self.buckets):
            b = self.buckets[self._next_launch]
            if b.n_ready < len(b.params):
                break
            self._launch(b)
            self._next_launch += 1

    def _launch(self, b: _Bucket):
        b.launched = True
        self._tp_due = True   # new data-parallel sums: the TP completion of SP gradients is due again
        if self.world == 1:
            return
        g = self.grad_view(b)
        side = wgrad_stream(self.device)
        # The bucket's weight gradients may still be in flight on the wgrad side stream (parallel/linear.py):
        # issue the collective from that stream after it has also caught up with the compute stream, so RCCL
        # waits for both while the compute stream itself never blocks.
        ctx = contextlib.nullcontext()
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(self.device))
            ctx = torch.cuda.stream(side)
        with ctx:
            if self.shard:
                b.work = dist.reduce_scatter_tensor(self.grad_shard_view(b), g, op=dist.ReduceOp.SUM,
                                                    group=self.group, async_op=True)
            else:
                # a bucket below the group's measured crossover (typically the small tail bucket) takes the
                # direct-peer xGMI all-reduce on the stream (comm/custom_allreduce.py); the rest RCCL
                car = use_custom_allreduce(g, self.group)
                if car is not None:
                    car.all_reduce(g)
                    b.work = None
                else:
                    b.work = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _join_wgrad_stream(self):
        join_wgrad_stream(self.device)

    def _finalize_backward(self):
        self._callback_queued = False
        try:
            self._launch_remaining()
        finally:
            # every main_grad write of this backward is ordered before whatever the compute stream does next
            self._join_wgrad_stream()

    def _launch_remaining(self):
        self._join_opt_stream()   # the zero-fill below writes gradient buckets the last update may still read
        if not self._sync_enabled:
            for b in self.buckets:
                b.n_ready = 0
            return
        with torch.no_grad():
            for p in self.params:
                if not p._dph_accum:   # unused in this step: contribute zeros
                    p.main_grad.zero_()
        for b in self.buckets[self._next_launch:]:
            self._launch(b)
        self._next_launch = len(self.buckets)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no collective) -- for gradient accumulation micro-steps."""
        old = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = old

    def zero_grad(self):
        for p in self.params:
            p._dph_accum = False
            p.grad = None
        for b in self.buckets:
            b.n_ready = 0
            b.launched = False
        self._next_launch = 0

    # ------------------------------------------------------------------------------------------ optimizer
    def configure_optimizer(self, cfg: OptimConfig):
        self.opt_cfg = cfg
        n = self.master.numel()
        k = 2 if cfg.name == "adamw" else (1 if cfg.momentum else 0)
        self.opt_state = [torch.zeros(n, dtype=torch.float32, device=self.device) for _ in range(k)]
        if cfg.name == "sgd" and not cfg.momentum:
            self.opt_state = [torch.zeros(1, dtype=torch.float32, device=self.device)]
        self.step_count = 0

    def _wait_reduce(self, b):
        if b.work is not None:
            b.work.wait()
            b.work = None

    def _global_sumsq(self) -> torch.Tensor:
        for b in self.buckets:
            self._wait_reduce(b)
        src = self.grad_shard if self.shard else self.flat_grad
        sq = optim_ref.global_grad_norm([src]) ** 2
        if self.shard:
            dist.all_reduce(sq, group=self.group)
        return sq / (self.world * self.world)   # gradients are SUMs over ranks

    @torch.no_grad()
    def step(self, lr: Optional[float] = None):
        cfg = self.opt_cfg
        assert cfg is not None, "call configure_optimizer first"
        if lr is not None:
            cfg.lr = lr
        if not self._sync_enabled:
            raise RuntimeError("optimizer step inside no_sync()")
        self.step_count += 1
        if self._tp_partial:
            self.finish_grad_sync()
        else:
            check_xgmi_health()   # a stalled direct-peer all-reduce must stop training, not feed the update
        if cfg.max_grad_norm is not None:
            norm = self._global_sumsq().sqrt()
            self._gscale.copy_(torch.clamp(cfg.max_grad_norm / (norm + 1e-6), max=1.0) / self.world)
            self.last_grad_norm = norm
        else:
            self._gscale.fill_(1.0 / self.world)   # (a previous step may have clipped, or the guard poisoned it)
        if _car.active():
            # every reduction of the step (buckets, TP / SP all-reduces) is queued ahead of the guard, which skips the
            # update on every rank if any direct-peer barrier of the group timed out (comm/custom_allreduce.py)
            for b in self.buckets:
                self._wait_reduce(b)
            _car.guard_update(self._gscale)
        native = _lib.use_native(self.master)
        hyper = _hyper_for(self, native)
        b1, b2 = cfg.betas
        bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
        side = self._step_stream(cfg)
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(self.device))   # gradients (and the clip scale) are final
        # Sharded: update and re-gather in FORWARD order (buckets are laid out in backward order).  RCCL runs the
        # all-gathers in issue order, so the first layers' parameters arrive first and the next forward waits
        # for one bucket's all-gather instead of the whole chain.  The overlapped step takes the same order.
        order = list(reversed(self.buckets)) if (self.shard or side is not None) else self.buckets
        for b in order:
            with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
                self._wait_reduce(b)   # Work.wait() orders the stream current at the call
                self._update_bucket(b, cfg, native, hyper, b1, b2, bc1, bc2)
                if self.shard:
                    full = self.param_view(b)
                    pout = self.param_shard_view(b)
                    src = pout.clone() if self.is_gloo else pout
                    b.ag_work = dist.all_gather_into_tensor(full, src, group=self.group, async_op=True)
                elif side is not None:
                    b.opt_event = torch.cuda.Event()
                    b.opt_event.record(side)

    def _step_stream(self, cfg: OptimConfig):
        """The side stream of an overlapped optimizer step, or None (CPU, capturable / graph-captured steps)."""
        if not self.overlap_step or cfg.capturable or torch.cuda.is_current_stream_capturing():
            return None
        if self._opt_stream is None:
            self._opt_stream = torch.cuda.Stream(device=self.device)
        return self._opt_stream

    def _join_opt_stream(self):
        if self._opt_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
            for b in self.buckets:
                b.opt_event = None

    def _update_bucket(self, b: _Bucket, cfg: OptimConfig, native: bool, hyper, b1, b2, bc1, bc2):
        master = self.master_view(b)
        grad = self.grad_shard_view(b)
        pout = self.param_shard_view(b)
        sl = self.opt_slice(b)
        if cfg.name == "adamw":
            m, v = self.opt_state[0][sl], self.opt_state[1][sl]
            if native:
                _lib.ops().adamw_step_(master, m, v, grad, pout, cfg.lr, b1, b2, cfg.eps, cfg.weight_decay,
                                       bc1, bc2, self._gscale, hyper=hyper)
            else:
                optim_ref.adamw_reference_(master, m, v, grad, cfg.lr, b1, b2, cfg.eps, cfg.weight_decay, bc1,
                                           bc2, self._gscale)
                pout.copy_(master)
        else:
            buf = self.opt_state[0][sl] if cfg.momentum else self.opt_state[0]
            if native:
                _lib.ops().sgd_step_(master, buf, grad, pout, cfg.lr, cfg.momentum, cfg.dampening,
                                     cfg.weight_decay, cfg.nesterov, self.step_count == 1, self._gscale,
                                     hyper=hyper)
            else:
                optim_ref.sgd_reference_(master, buf, grad, cfg.lr, cfg.momentum, cfg.dampening,
                                         cfg.weight_decay, cfg.nesterov, self.step_count == 1, self._gscale)
                pout.copy_(master)

    def _wait_ag(self, ids, module=None, args=None):
        # Wait for the module's buckets AND every bucket before them in forward order (higher index): the
        # all-gathers were issued in that order, so on RCCL this costs nothing extra, and a parameter that some
        # earlier module reads functionally (outside its own forward) is covered as well.
        ids = list(ids)
        if not ids:
            return
        for i in range(len(self.buckets) - 1, min(ids) - 1, -1):
            b = self.buckets[i]
            if b.ag_work is not None:
                b.ag_work.wait()
                b.ag_work = None
            if b.opt_event is not None:
                torch.cuda.current_stream(self.device).wait_event(b.opt_event)
                b.opt_event = None

    def synchronize(self):
        """Wait for every outstanding collective (end of step / before checkpointing or evaluation)."""
        self.finish_grad_sync()
        self._wait_ag(range(len(self.buckets)))
        self._join_opt_stream()

    # ------------------------------------------------------------------------------------------ state
    # checkpoint protocol shared with fsdp.ZeRO3Engine (utils/checkpointing.py): ``groups`` are the buckets, each a
    # padded flat vector of its parameters; this rank's optimizer-side slice of bucket b is ``opt_slice(b)``.
    @property
    def groups(self):
        return self.buckets

    @property
    def sharded_state(self) -> bool:
        return self.shard

    def opt_slice(self, b: _Bucket) -> slice:
        if self.shard:
            return slice(b.shard_offset, b.shard_offset + b.shard_numel)
        return slice(b.offset, b.offset + b.numel)

    @torch.no_grad()
    def refresh_params_from_master(self):
        """After the fp32 master changed outside ``step`` (checkpoint load): parameters <- master (re-gathered
        across the group when sharded)."""
        self.synchronize()
        for b in self.buckets:
            self.param_shard_view(b).copy_(self.master_view(b))
            if self.shard:
                dist.all_gather_into_tensor(self.param_view(b), self.param_shard_view(b).clone(), group=self.group)

    @torch.no_grad()
    def load_full_state_dict(self, sd: dict):
        """Full model state (parameters live in the flat buffer, so the module loads in place); the fp32 master is
        re-derived from the loaded parameters (a following optimizer-state load overrides it)."""
        self.synchronize()
        self.module.load_state_dict(sd)
        for b in self.buckets:
            self.master_view(b).copy_(self.param_shard_view(b))

    def optimizer_state_dict(self) -> dict:
        """Rank-local optimizer state (the shard when sharded) + layout metadata."""
        self.synchronize()
        return {"step": self.step_count, "master": self.master.cpu(),
                "state": [s.cpu() for s in self.opt_state], "world": self.world, "rank": self.rank,
                "shard": self.shard, "total": self.total, "kind": "dp",
                # unpadded length of every bucket: lets a resume with another bucket partition re-cut the state
                "group_real": [sum(align_up(p.numel()) for p in b.params) for b in self.buckets]}

    def load_optimizer_state_dict(self, sd: dict):
        assert sd.get("kind", "dp") == "dp" and sd["total"] == self.total and sd["shard"] == self.shard and \
            sd["world"] == self.world, \
            "optimizer state layout mismatch (another world size or engine: use utils.checkpointing)"
        self.step_count = int(sd["step"])
        with torch.no_grad():
            self.master.copy_(sd["master"])
            for s, t in zip(self.opt_state, sd["state"]):
                s.copy_(t)
        self.refresh_params_from_master()


class _EngineOptimizer:
    """torch.optim-like facade over DataParallelEngine (step / zero_grad / param_groups[lr])."""

    def __init__(self, engine: DataParallelEngine, cfg: OptimConfig):
        self.engine = engine
        engine.configure_optimizer(cfg)
        self.param_groups = [{"lr": cfg.lr}]

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.engine.step(lr=self.param_groups[0]["lr"])
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.engine.zero_grad()

    def state_dict(self):
        return self.engine.optimizer_state_dict()

    def load_state_dict(self, sd):
        self.engine.load_optimizer_state_dict(sd)


class DistributedDataParallel(nn.Module):
    """Bucketed all-reduce data parallelism (replicated optimizer state).

    ``DDP(model)`` mirrors ``torch.nn.parallel.DistributedDataParallel(model, device_ids=[local_rank])``:
    parameters are broadcast from rank 0 at construction and gradients are SUM-reduced (the 1/world mean is
    applied inside the optimizer kernel).  Create the optimizer with ``ddp.make_optimizer(...)``.
    """

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 256.0,
                 mixed_precision: Optional[MixedPrecision] = None, overlap: bool = True,
                 broadcast_buffers: bool = True, **_ignored):
        super().__init__()
        self.module = module
        self.engine = DataParallelEngine(module, process_group, shard=False, mixed_precision=mixed_precision,
                                         bucket_cap_mb=bucket_cap_mb, overlap=overlap)
        self.process_group = process_group
        # torch DDP default: module buffers (BatchNorm running stats) follow rank 0 at every training forward
        self.broadcast_buffers = broadcast_buffers and self.engine.world > 1 and any(True for _ in module.buffers())

    @torch.no_grad()
    def _sync_buffers(self):
        """One coalesced broadcast per buffer dtype from rank 0 of the group."""
        src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
        by_dtype: dict = {}
        for b in self.module.buffers():
            by_dtype.setdefault(b.dtype, []).append(b)
        for bufs in by_dtype.values():
            flat = torch.cat([b.reshape(-1) for b in bufs])
            dist.broadcast(flat, src=src, group=self.process_group)
            o = 0
            for b in bufs:
                b.copy_(flat[o:o + b.numel()].view_as(b))
                o += b.numel()

    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.module.training:
            self._sync_buffers()
        return self.module(*args, **kwargs)

    def make_optimizer(self, name: str = "adamw", **kw) -> _EngineOptimizer:
        return _EngineOptimizer(self.engine, OptimConfig(name=name, **kw))

    def no_sync(self):
        return self.engine.no_sync()

    def synchronize(self):
        self.engine.synchronize()


DDP = DistributedDataParallel
