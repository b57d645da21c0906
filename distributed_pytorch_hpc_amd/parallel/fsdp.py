"""Fully-sharded data parallelism (FSDP) with the reference's four sharding strategies.

Capability parity with scripts/02_fully_sharded_fsdp/resnet_fsdp_training.py:193-212 and multinode_fsdp_unet.py:202-298
(``FSDP(model, auto_wrap_policy=size_based_auto_wrap_policy(min_num_params=1e5), sharding_strategy=FULL_SHARD,
mixed_precision=MixedPrecision(bf16, bf16, bf16))`` + FULL_STATE_DICT rank-0 consolidation) and with FSDP2
``fully_shard`` on a dp mesh (fsdp_tp/fsdp_tp_example.py:187), including the per-block wrapping the reference only
documents (ModuleWrapPolicy({TransformerBlock}), X8).

    FSDP(module, sharding_strategy=..., auto_wrap_policy=..., mixed_precision=..., process_group=...)

  NO_SHARD       -> DataParallelEngine(shard=False): bucketed all-reduce (DDP)
  SHARD_GRAD_OP  -> DataParallelEngine(shard=True):  reduce-scatter grads, sharded fp32 optimizer state, parameters
                    all-gathered after the step and kept resident (ZeRO-2; the default choice on a 288 GB MI355X:
                    Llama-2-7B's full bf16 parameters are 13.5 GB, so resharding buys little and costs a second
                    all-gather per step)
  FULL_SHARD     -> ZeRO3Engine: only the 1/N parameter shard persists; each wrapped unit is all-gathered right
                    before its forward and again before its backward (next unit prefetched asynchronously) and
                    freed after use; gradients are reduce-scattered per unit as soon as the unit's backward is done
  HYBRID_SHARD   -> FULL_SHARD inside ``process_group`` (the node) + all-reduce of the gradient shards across
                    ``replicate_group`` (other nodes); on a single node it is FULL_SHARD.
Create the optimizer with ``fsdp.make_optimizer("adamw", lr=...)`` (fused CDNA4 kernel on the local shard).
"""
from __future__ import annotations

import contextlib
import os
from enum import Enum
from functools import partial
from typing import Callable, Iterable, Optional

import torch
import torch.distributed as dist
from torch import nn

from ..comm import custom_allreduce as _car
from ..comm.custom_allreduce import check_health as check_xgmi_health
from ..ops import _lib
from ..train import optim as optim_ref
from ..utils.flat import ALIGN, align_up, flat_order, flat_order_like, param_view
from .data_parallel import DataParallelEngine, MixedPrecision, OptimConfig, _EngineOptimizer, _hyper_for
from .linear import convert_linears_, join_wgrad_stream


class ShardingStrategy(Enum):
    FULL_SHARD = "FULL_SHARD"
    SHARD_GRAD_OP = "SHARD_GRAD_OP"
    NO_SHARD = "NO_SHARD"
    HYBRID_SHARD = "HYBRID_SHARD"


# ------------------------------------------------------------------------------------------------ wrap policies
def size_based_auto_wrap_policy(min_num_params: int = int(1e5)) -> Callable:
    def policy(module: nn.Module, unwrapped_params: int) -> bool:
        return unwrapped_params >= min_num_params
    policy.min_num_params = min_num_params
    return policy


def ModuleWrapPolicy(classes: Iterable[type]) -> Callable:  # noqa: N802 - torch-compatible name
    classes = tuple(classes)

    def policy(module: nn.Module, unwrapped_params: int) -> bool:
        return isinstance(module, classes)
    return policy


def _select_units(root: nn.Module, policy: Optional[Callable]) -> list[nn.Module]:
    """Post-order: a module becomes a unit if the policy accepts it given the params not already owned by
    nested units; the root is always the last unit."""
    units: list[nn.Module] = []
    owned: set[int] = set()

    def visit(m):
        for c in m.children():
            visit(c)
        if m is root or policy is None or isinstance(m, (nn.ModuleList, nn.ModuleDict)):
            return   # containers have no forward of their own: their params stay with the enclosing unit
        free = [p for p in m.parameters() if p.requires_grad and id(p) not in owned]
        n = sum(p.numel() for p in free)
        if n and policy(m, n):
            units.append(m)
            owned.update(id(p) for p in free)

    visit(root)
    units.append(root)
    return units


# ------------------------------------------------------------------------------------------------ ZeRO-3 engine
class _Unit:
    def __init__(self, idx, module, params):
        self.idx, self.module, self.params = idx, module, params
        self.numel = self.shard_numel = self.shard_offset = 0
        self.full = self.grad_full = None
        self.gathered = False
        self.ag_work = self.rs_work = None
        self.n_ready = 0
        self.launched = False


def _free(t: torch.Tensor):
    if t.untyped_storage().size() != 0:
        t.untyped_storage().resize_(0)


def _alloc(t: torch.Tensor):
    need = t.numel() * t.element_size()
    if t.untyped_storage().size() != need:
        t.untyped_storage().resize_(need)


class ZeRO3Engine:
    def __init__(self, module: nn.Module, process_group=None, mixed_precision: Optional[MixedPrecision] = None,
                 auto_wrap_policy: Optional[Callable] = None, reshard_after_forward: bool = True,
                 replicate_group=None, prefetch: bool = True):
        self.module, self.group, self.replicate_group = module, process_group, replicate_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.reshard = reshard_after_forward
        self.prefetch = prefetch
        mp = mixed_precision or MixedPrecision()
        if mp.param_dtype is not None:
            for p in module.parameters():
                p.data = p.data.to(mp.param_dtype)
        if mp.buffer_dtype is not None:
            for b in module.buffers():
                if b.is_floating_point():
                    b.data = b.data.to(mp.buffer_dtype)
        convert_linears_(module)
        units_m = _select_units(module, auto_wrap_policy)
        owned, self.units = set(), []
        for m in units_m:
            ps = [p for p in m.parameters() if p.requires_grad and id(p) not in owned]
            owned.update(id(p) for p in ps)
            if ps:
                self.units.append(_Unit(len(self.units), m, ps))
        params = [p for u in self.units for p in u.params]
        self.params = params
        self.param_dtype = params[0].dtype
        self.device = params[0].device
        self.grad_dtype = mp.reduce_dtype or self.param_dtype
        self.is_gloo = dist.is_initialized() and dist.get_backend(process_group) == "gloo"
        soff = 0
        for u in self.units:
            u.numel = align_up(sum(align_up(p.numel()) for p in u.params), ALIGN * self.world)
            u.shard_numel = u.numel // self.world
            u.shard_offset = soff
            soff += u.shard_numel
        self.shard_total = soff
        self.param_shard = torch.zeros(soff, dtype=self.param_dtype, device=self.device)
        self.grad_shard = torch.zeros(soff, dtype=self.grad_dtype, device=self.device)
        # A shard group of one: a unit's gathered parameters / full gradient ARE its shard, so they alias the shard
        # buffers -- the all-gather, reduce-scatter and free of the general path degenerate to nothing instead of a
        # copy each (3 per unit per step) and an allocator round trip.  Same engine, same update order as world > 1.
        self._alias = self.world == 1
        self._unit_of = {}
        with torch.no_grad():
            for u in self.units:
                full = torch.zeros(u.numel, dtype=self.param_dtype, device=self.device)
                o = 0
                for p in u.params:
                    n = p.numel()
                    full[o:o + n].copy_(flat_order(p.data))
                    o += align_up(n)
                if self.world > 1:   # every rank starts from rank 0's weights
                    src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
                    dist.broadcast(full, src=src, group=process_group)
                self.shard_view(u).copy_(full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel])
                if self._alias:
                    u.full, u.grad_full = self.shard_view(u), self.grad_shard_view(u)
                else:
                    u.full = full
                    u.grad_full = torch.zeros(u.numel, dtype=self.grad_dtype, device=self.device)
                o = 0
                for p in u.params:
                    n = p.numel()
                    p.main_grad = param_view(u.grad_full[o:o + n], p)   # channels-last weights stay so
                    p.data = param_view(u.full[o:o + n], p)
                    p._dph_accum = False
                    p._dph_grad_ready = partial(self._on_grad_ready, p)
                    self._unit_of[id(p)] = u
                    o += align_up(n)
                u.gathered = True
        self.master = self.param_shard.float()
        self.opt_state: list[torch.Tensor] = []
        self.opt_cfg: Optional[OptimConfig] = None
        self.step_count = 0
        self._hyper = None
        self._gscale = torch.full((1,), 1.0 / self._dp_world(), dtype=torch.float32, device=self.device)
        self._sync_enabled = True
        self._callback_queued = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._post_accumulate) for p in params]
        for u in self.units:
            u.module.register_forward_pre_hook(partial(self._pre_forward, u))
            u.module.register_forward_hook(partial(self._post_forward, u))
            u.module.register_full_backward_pre_hook(partial(self._pre_backward, u))
        for u in self.units:
            self._release(u)   # only shards persist from here on

    def _dp_world(self):
        w = self.world
        if self.replicate_group is not None:
            w *= dist.get_world_size(self.replicate_group)
        return w

    def shard_view(self, u):
        return self.param_shard[u.shard_offset:u.shard_offset + u.shard_numel]

    def grad_shard_view(self, u):
        return self.grad_shard[u.shard_offset:u.shard_offset + u.shard_numel]

    def master_view(self, u):
        return self.master[u.shard_offset:u.shard_offset + u.shard_numel]

    # ---------------------------------------------------------------------------------------- gather / free
    def _start_gather(self, u):
        if u.gathered or u.ag_work is not None:
            return
        if self._alias:
            u.gathered = True
            return
        _alloc(u.full)
        if self.world == 1:
            u.full.copy_(self.shard_view(u))
            u.gathered = True
            return
        src = self.shard_view(u)
        if self.is_gloo:
            src = src.clone()
        u.ag_work = dist.all_gather_into_tensor(u.full, src, group=self.group, async_op=True)

    def _gather(self, u):
        self._start_gather(u)
        if u.ag_work is not None:
            u.ag_work.wait()
            u.ag_work = None
        u.gathered = True

    def _release(self, u):
        if self._alias or (u is self.units[-1] and not self.reshard):
            return
        if u.ag_work is not None:
            u.ag_work.wait()
            u.ag_work = None
        _free(u.full)
        u.gathered = False

    # ---------------------------------------------------------------------------------------- hooks
    def _pre_forward(self, u, module, args):
        self._gather(u)
        if self.prefetch and u.idx + 1 < len(self.units) - 1:
            self._start_gather(self.units[u.idx + 1])

    def _post_forward(self, u, module, args, out):
        # reshard after forward (the backward pre-hook gathers again); the root unit stays resident
        if self.reshard and u is not self.units[-1]:
            self._release(u)

    def _pre_backward(self, u, module, grad_out):
        self._gather(u)
        # a freshly allocated full gradient holds garbage (its padding included); an aliased one is the shard, whose
        # padding was zeroed at construction and is never written, and every parameter slice in it is either written
        # by this backward or zeroed in _launch -- so only the non-aliased buffer needs the fill
        if not self._alias:
            _alloc(u.grad_full)
            if not any(p._dph_accum for p in u.params):
                u.grad_full.zero_()
        if self.prefetch and u.idx >= 1 and u.idx - 1 < len(self.units) - 1:
            self._start_gather(self.units[u.idx - 1])

    def _post_accumulate(self, p):
        g = p.grad
        if g is None:
            return
        u = self._unit_of[id(p)]
        if not self._alias:
            _alloc(u.grad_full)
        with torch.no_grad():
            if p._dph_accum:
                p.main_grad.add_(g)
            else:
                p.main_grad.copy_(g)
                p._dph_accum = True
        p.grad = None
        self._on_grad_ready(p)

    def _on_grad_ready(self, p):
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
        u = self._unit_of[id(p)]
        u.n_ready += 1
        if u.n_ready == len(u.params) and self._sync_enabled:
            self._launch(u)

    def _join_wgrad_stream(self):
        # weight-gradient GEMMs into u.grad_full may run on the wgrad side stream (parallel/linear.py); the unit's
        # buffer is zero-filled, reduce-scattered and freed on the compute stream, so order it after them
        join_wgrad_stream(self.device)

    def _launch(self, u):
        if u.launched:
            return
        u.launched = True
        self._join_wgrad_stream()
        with torch.no_grad():
            for p in u.params:
                if not p._dph_accum:
                    p.main_grad.zero_()
        if self._alias:
            pass   # the full gradient is the shard
        elif self.world == 1:
            self.grad_shard_view(u).copy_(u.grad_full)
        else:
            u.rs_work = dist.reduce_scatter_tensor(self.grad_shard_view(u), u.grad_full, op=dist.ReduceOp.SUM,
                                                   group=self.group, async_op=True)
        if u is not self.units[-1]:
            self._release(u)

    def _finalize_backward(self):
        self._callback_queued = False
        self._join_wgrad_stream()
        if not self._sync_enabled:
            for u in self.units:
                u.n_ready = 0
            return
        if not self._alias:
            _alloc(self.units[-1].grad_full)
        for u in self.units:
            if not u.launched:
                if not self._alias:
                    _alloc(u.grad_full)
                self._launch(u)
        for u in self.units:
            if u.rs_work is not None:
                u.rs_work.wait()
                u.rs_work = None
            if not self._alias:
                _free(u.grad_full)
        if self.replicate_group is not None:
            dist.all_reduce(self.grad_shard, group=self.replicate_group)

    @contextlib.contextmanager
    def no_sync(self):
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
        for u in self.units:
            u.n_ready = 0
            u.launched = False

    # ---------------------------------------------------------------------------------------- optimizer
    def configure_optimizer(self, cfg: OptimConfig):
        self.opt_cfg = cfg
        k = 2 if cfg.name == "adamw" else 1
        self.opt_state = [torch.zeros_like(self.master) for _ in range(k)]
        self.step_count = 0

    @torch.no_grad()
    def step(self, lr: Optional[float] = None):
        cfg = self.opt_cfg
        if lr is not None:
            cfg.lr = lr
        self.step_count += 1
        check_xgmi_health()   # TP / SP all-reduces of this step may have used the direct-peer path
        if cfg.max_grad_norm is not None:
            sq = optim_ref.global_grad_norm([self.grad_shard]) ** 2
            if self.world > 1:
                dist.all_reduce(sq, group=self.group)
            norm = sq.sqrt() / self._dp_world()
            self._gscale.copy_(torch.clamp(cfg.max_grad_norm / (norm + 1e-6), max=1.0) / self._dp_world())
        if _car.active():
            if cfg.max_grad_norm is None:
                self._gscale.fill_(1.0 / self._dp_world())   # a previous step's guard may have poisoned it
            _car.guard_update(self._gscale)   # skip the update on every rank if a direct-peer barrier timed out
        native = _lib.use_native(self.master)
        hyper = _hyper_for(self, native)
        b1, b2 = cfg.betas
        bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
        if cfg.name == "adamw":
            m, v = self.opt_state
            if native:
                _lib.ops().adamw_step_(self.master, m, v, self.grad_shard, self.param_shard, cfg.lr, b1, b2, cfg.eps,
                                       cfg.weight_decay, bc1, bc2, self._gscale, hyper=hyper)
            else:
                optim_ref.adamw_reference_(self.master, m, v, self.grad_shard, cfg.lr, b1, b2, cfg.eps,
                                           cfg.weight_decay, bc1, bc2, self._gscale)
                self.param_shard.copy_(self.master)
        else:
            buf = self.opt_state[0]
            if native:
                _lib.ops().sgd_step_(self.master, buf, self.grad_shard, self.param_shard, cfg.lr, cfg.momentum,
                                     cfg.dampening, cfg.weight_decay, cfg.nesterov, self.step_count == 1, self._gscale,
                                     hyper=hyper)
            else:
                optim_ref.sgd_reference_(self.master, buf, self.grad_shard, cfg.lr, cfg.momentum, cfg.dampening,
                                         cfg.weight_decay, cfg.nesterov, self.step_count == 1, self._gscale)
                self.param_shard.copy_(self.master)
        # resident units (root when not resharding) must see the update
        for u in self.units:
            if u.gathered:
                u.gathered = False
                self._gather(u)

    def synchronize(self):
        for u in self.units:
            if u.ag_work is not None:
                u.ag_work.wait()
                u.ag_work = None

    # ---------------------------------------------------------------------------------------- state
    # checkpoint protocol shared with DataParallelEngine (utils/checkpointing.py): ``groups`` are the units, each a
    # padded flat vector of its parameters; this rank's optimizer-side slice of unit u is ``opt_slice(u)``.
    sharded_state = True

    @property
    def groups(self):
        return self.units

    def opt_slice(self, u) -> slice:
        return slice(u.shard_offset, u.shard_offset + u.shard_numel)

    def full_state_dict(self, rank0_only: bool = True, offload_to_cpu: bool = True) -> dict:
        """FULL_STATE_DICT consolidation (multinode_fsdp_unet.py:285-291): gather every unit, copy out, free.
        Collective over the shard group; with ``rank0_only`` only group rank 0 makes (and returns) the copies."""
        keep = not rank0_only or self.rank == 0
        out = {}
        names = {id(p): n for n, p in self.module.named_parameters()}
        for u in self.units:
            was = u.gathered
            self._gather(u)
            if keep:
                for p in u.params:
                    t = p.detach()
                    out[names[id(p)]] = t.cpu().clone() if offload_to_cpu else t.clone()
            if not was:
                self._release(u)
        if not keep:
            return {}
        for n, b in self.module.named_buffers():
            out[n] = b.detach().cpu().clone() if offload_to_cpu else b.detach().clone()
        return out

    @torch.no_grad()
    def load_full_state_dict(self, sd: dict):
        """Inverse of ``full_state_dict``: every rank passes the same full (unsharded) state; each unit's padded
        vector is rebuilt from it and this rank keeps its 1/N slice (parameter shard + fp32 master).  Buffers are
        copied into the module.  Released units are never written through the module's (freed) parameters."""
        names = {id(p): n for n, p in self.module.named_parameters()}
        missing = [names[id(p)] for p in self.params if names[id(p)] not in sd]
        if missing:
            raise KeyError(f"load_full_state_dict: missing parameters {missing[:4]}")
        for u in self.units:
            full = torch.zeros(u.numel, dtype=self.param_dtype)
            o = 0
            for p in u.params:
                n = p.numel()
                full[o:o + n].copy_(flat_order_like(sd[names[id(p)]], p, names[id(p)]))
                o += align_up(n)
            mine = full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel].to(self.device)
            self.shard_view(u).copy_(mine)
            self.master_view(u).copy_(mine.float())
        for n, b in self.module.named_buffers():
            if n in sd:
                b.copy_(sd[n])
        self.refresh_params_from_master(cast=False)

    @torch.no_grad()
    def refresh_params_from_master(self, cast: bool = True):
        """After the fp32 master changed outside ``step`` (checkpoint load): parameter shard <- master, and the
        resident (gathered) units are re-gathered so the module sees the new values."""
        self.synchronize()
        if cast:
            self.param_shard.copy_(self.master)
        for u in self.units:
            if u.gathered:
                u.gathered = False
                self._gather(u)

    def optimizer_state_dict(self):
        self.synchronize()
        return {"step": self.step_count, "master": self.master.cpu(), "state": [s.cpu() for s in self.opt_state],
                "world": self.world, "rank": self.rank, "shard": True, "total": self.shard_total * self.world,
                "kind": "zero3", "group_real": [sum(align_up(p.numel()) for p in u.params) for u in self.units]}

    def load_optimizer_state_dict(self, sd):
        assert sd.get("kind") == "zero3" and sd["world"] == self.world and \
            sd["total"] == self.shard_total * self.world, \
            "optimizer state layout mismatch (another world size or engine: use utils.checkpointing)"
        self.step_count = int(sd["step"])
        self.master.copy_(sd["master"])
        for s, t in zip(self.opt_state, sd["state"]):
            s.copy_(t)
        self.refresh_params_from_master()


# ------------------------------------------------------------------------------------------------ module wrapper
class FullyShardedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None,
                 sharding_strategy: ShardingStrategy | str = ShardingStrategy.FULL_SHARD,
                 mixed_precision: Optional[MixedPrecision] = None, auto_wrap_policy: Optional[Callable] = None,
                 bucket_cap_mb: float = 256.0, reshard_after_forward: bool = True, replicate_group=None,
                 device_id=None, **_ignored):
        super().__init__()
        if isinstance(sharding_strategy, str):
            sharding_strategy = ShardingStrategy(sharding_strategy)
        self.module = module
        self.strategy = sharding_strategy
        if sharding_strategy == ShardingStrategy.NO_SHARD:
            self.engine = DataParallelEngine(module, process_group, shard=False, mixed_precision=mixed_precision,
                                             bucket_cap_mb=bucket_cap_mb)
        elif sharding_strategy == ShardingStrategy.SHARD_GRAD_OP:
            self.engine = DataParallelEngine(module, process_group, shard=True, mixed_precision=mixed_precision,
                                             bucket_cap_mb=bucket_cap_mb)
        else:
            self.engine = ZeRO3Engine(module, process_group, mixed_precision, auto_wrap_policy,
                                      reshard_after_forward=reshard_after_forward,
                                      replicate_group=replicate_group if sharding_strategy ==
                                      ShardingStrategy.HYBRID_SHARD else None)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def make_optimizer(self, name: str = "adamw", **kw) -> _EngineOptimizer:
        return _EngineOptimizer(self.engine, OptimConfig(name=name, **kw))

    def no_sync(self):
        return self.engine.no_sync()

    def state_dict(self, *args, **kwargs):
        """Unsharded parameters (gathered unit by unit: a FULL_SHARD model's released storage is never read)."""
        return self.full_state_dict(rank0_only=False, offload_to_cpu=True)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Full (unsharded) state as returned by ``state_dict``; every rank passes the same one.  Missing parameters
        always raise; with ``strict`` keys the module does not have raise too."""
        if strict:
            known = set(self.module.state_dict().keys()) if not isinstance(self.engine, ZeRO3Engine) else \
                {n for n, _ in self.module.named_parameters()} | {n for n, _ in self.module.named_buffers()}
            extra = sorted(set(state_dict) - known)
            if extra:
                raise KeyError(f"load_state_dict: unexpected keys {extra[:4]}")
        self.engine.load_full_state_dict(state_dict)

    def full_state_dict(self, rank0_only: bool = True, offload_to_cpu: bool = True) -> dict:
        if isinstance(self.engine, ZeRO3Engine):
            return self.engine.full_state_dict(rank0_only, offload_to_cpu)
        self.engine.synchronize()
        rank = dist.get_rank() if dist.is_initialized() else 0
        if rank0_only and rank != 0:
            return {}
        return {k: (v.detach().cpu().clone() if offload_to_cpu else v.detach().clone())
                for k, v in self.module.state_dict().items()}


FSDP = FullyShardedDataParallel


def fully_shard(module: nn.Module, mesh_group=None, reshard_after_forward: bool = True,
                mp_policy: Optional[MixedPrecision] = None, block_types: Iterable[type] = ()) -> FullyShardedDataParallel:
    """FSDP2-style entry point (fsdp_tp_example.py:187): shard ``module`` over the dp group, one unit per block
    of ``block_types`` (per-block sharding instead of the reference's root-only unit)."""
    policy = ModuleWrapPolicy(block_types) if block_types else None
    return FullyShardedDataParallel(module, mesh_group, ShardingStrategy.FULL_SHARD, mp_policy, policy,
                                    reshard_after_forward=reshard_after_forward)
