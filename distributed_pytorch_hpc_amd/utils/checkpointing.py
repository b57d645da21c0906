"""Checkpoint / resume for every parallel layout of the framework.

Reference capability: utils/checkpointing.py:23-88 (rank-0 save of model+optimizer+epoch, barrier, load with
map_location), the DDP ``snapshot.pt`` auto-resume (scripts/01_data_parallel_ddp/multinode_ddp_basic.py:144-196)
and the FSDP FULL_STATE_DICT rank-0 consolidation (scripts/02_fully_sharded_fsdp/multinode_fsdp_unet.py:282-298).
Fixes the reference defects X15 (one module used everywhere; a single writer per job, not per node).

Two formats:
  * ``save_checkpoint`` / ``load_checkpoint``: consolidated single file written by global rank 0 (small models,
    interoperability).  Every rank must call both.  With an engine-backed model (DDP / FSDP / ZeRO engines of
    parallel/) the model state is the FULL state -- gathered unit by unit for FULL_SHARD, whose module parameters
    point at released storage -- and the optimizer state is stored per parameter name in the logical tensor shape
    (``format: "full"``), so a file loads into any strategy and any data-parallel world size.
  * ``ShardedCheckpointer``: one directory per step, ``rank{r}.pt`` per rank holding that rank's model shard
    (TP/PP shards; data-parallel replicas are written by their dp-rank-0 only; FULL_SHARD writes the gathered full
    state from dp-rank 0) and optimizer shard (the engine's fp32 master / m / v slice) + ``meta.json``.  Loading at
    a DIFFERENT data-parallel world size re-slices the engine's flat optimizer state (``reshard_engine_state``).
Both store the step/epoch, torch + HIP RNG state and arbitrary extra metadata; files are loaded with
``weights_only=True`` (tensors, numbers, strings, lists, dicts only).

Engines implement a small protocol (parallel/data_parallel.py, parallel/fsdp.py): ``groups`` (buckets / units:
padded flat vectors of ``.params``), ``opt_slice(g)`` (this rank's slice of g in master / optimizer state),
``sharded_state``, ``refresh_params_from_master()``, ``load_full_state_dict(sd)``.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Optional

import torch
import torch.distributed as dist

from .flat import ALIGN, align_up, flat_order_like, param_view


def _rank():
    return dist.get_rank() if dist.is_initialized() else 0


def _barrier():
    if dist.is_initialized():
        dist.barrier()


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def _engine_of(model, optimizer=None):
    """The framework engine behind ``optimizer`` (``make_optimizer`` facade) or ``model`` (DDP / FSDP wrapper)."""
    for o in (optimizer, model):
        e = getattr(o, "engine", None)
        if e is not None and hasattr(e, "groups"):
            return e
    return None


def rng_state() -> dict:
    st = {"torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: dict):
    if "torch" in st:
        torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


# ------------------------------------------------------------------------------------------------ engine state
def _rank_slice(engine, g) -> slice:
    """This rank's part of group g's padded full vector."""
    if engine.sharded_state:
        return slice(engine.rank * g.shard_numel, (engine.rank + 1) * g.shard_numel)
    return slice(0, g.numel)


def _state_vectors(engine) -> list[torch.Tensor]:
    """fp32 master + the optimizer-state vectors laid out like it (SGD without momentum keeps a dummy)."""
    n = engine.master.numel()
    return [engine.master] + [s for s in engine.opt_state if s.numel() == n]


def _gather_group(engine, vec: torch.Tensor, g) -> torch.Tensor:
    local = vec[engine.opt_slice(g)]
    if not engine.sharded_state or engine.world == 1:
        return local
    full = torch.empty(g.numel, dtype=vec.dtype, device=vec.device)
    dist.all_gather_into_tensor(full, local.clone() if engine.is_gloo else local, group=engine.group)
    return full


def full_model_state(model, engine=None) -> dict:
    """Unsharded model state (CPU) on global rank 0, ``{}`` elsewhere.  Collective when the parameters are sharded
    (FULL_SHARD gathers unit by unit) -- call it on every rank."""
    engine = engine if engine is not None else _engine_of(model)
    if engine is not None and hasattr(engine, "full_state_dict"):
        return engine.full_state_dict(rank0_only=True, offload_to_cpu=True)   # kept on the group's rank 0
    if engine is not None:
        engine.synchronize()   # sharded (ZeRO-2) parameter all-gathers still in flight
    if _rank() != 0:
        return {}
    return {k: v.detach().cpu().clone() for k, v in _unwrap(model).state_dict().items()}


def full_optimizer_state(engine) -> dict:
    """Layout-independent optimizer state: fp32 master and every state vector, per parameter NAME in the
    parameter's logical shape.  Collective over the engine's group; the dict is returned on group rank 0 only."""
    engine.synchronize()
    names = {id(p): n for n, p in engine.module.named_parameters()}
    vecs = _state_vectors(engine)
    keep = engine.rank == 0
    tensors: list[dict] = [{} for _ in vecs]
    for g in engine.groups:
        for k, vec in enumerate(vecs):
            full = _gather_group(engine, vec, g)
            if not keep:
                continue
            o = 0
            for p in g.params:
                n = p.numel()
                tensors[k][names[id(p)]] = param_view(full[o:o + n], p).contiguous().cpu().clone()
                o += align_up(n)
    if not keep:
        return {}
    cfg = engine.opt_cfg
    return {"format": "full", "step": int(engine.step_count), "optimizer": cfg.name if cfg else None,
            "master": tensors[0], "state": tensors[1:]}


@torch.no_grad()
def load_full_optimizer_state(engine, sd: dict):
    """Inverse of ``full_optimizer_state`` for any engine / world size (every rank passes the same dict)."""
    names = {id(p): n for n, p in engine.module.named_parameters()}
    vecs = _state_vectors(engine)
    srcs = [sd["master"]] + list(sd["state"])
    if len(srcs) != len(vecs):
        raise ValueError(f"optimizer state has {len(srcs) - 1} state vectors, the engine {len(vecs) - 1} "
                         f"(saved with optimizer {sd.get('optimizer')!r}?)")
    engine.synchronize()
    for g in engine.groups:
        rs = _rank_slice(engine, g)
        for src, vec in zip(srcs, vecs):
            full = torch.zeros(g.numel, dtype=torch.float32)
            o = 0
            for p in g.params:
                n = p.numel()
                full[o:o + n].copy_(flat_order_like(src[names[id(p)]], p, names[id(p)]))
                o += align_up(n)
            vec[engine.opt_slice(g)].copy_(full[rs])
    engine.step_count = int(sd["step"])
    engine.refresh_params_from_master()


def _load_model_state(model, engine, sd: dict):
    if engine is not None:
        engine.load_full_state_dict(sd)
    else:
        _unwrap(model).load_state_dict(sd)


# ------------------------------------------------------------------------------------------------ consolidated
def save_checkpoint(model, optimizer, epoch: int, path: str, extra: Optional[dict] = None, rank: Optional[int] = None):
    """Consolidated checkpoint written by global rank 0.  Every rank must call it (collective gathers for sharded
    engines, barrier at the end)."""
    rank = _rank() if rank is None else rank
    engine = _engine_of(model, optimizer)
    model_sd = full_model_state(model, engine)
    opt_sd = None
    if optimizer is not None:
        opt_sd = full_optimizer_state(engine) if engine is not None else \
            (optimizer.state_dict() if rank == 0 else None)
    if rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        state = {"model_state_dict": model_sd, "optimizer_state_dict": opt_sd, "epoch": int(epoch),
                 "rng": rng_state(), "extra": extra or {}}
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)   # atomic: a crash never leaves a truncated checkpoint
    _barrier()


def load_checkpoint(model, optimizer, path: str, device=None) -> int:
    """Restores model (+optimizer) in place on every rank; returns the stored epoch, or 0 when ``path`` is
    missing."""
    if not os.path.exists(path):
        return 0
    state = torch.load(path, map_location=device or "cpu", weights_only=True)
    engine = _engine_of(model, optimizer)
    _load_model_state(model, engine, state["model_state_dict"])
    osd = state.get("optimizer_state_dict")
    if optimizer is not None and osd is not None:
        if osd.get("format") == "full":
            if engine is None:
                raise ValueError("checkpoint holds a framework-engine optimizer state; build the optimizer with "
                                 "DDP/FSDP.make_optimizer to load it")
            load_full_optimizer_state(engine, osd)
        else:
            optimizer.load_state_dict(osd)
    if "rng" in state:
        set_rng_state(state["rng"])
    return int(state.get("epoch", 0))


# ------------------------------------------------------------------------------------------------ sharded
class ShardedCheckpointer:
    def __init__(self, root: str, model, engine=None, dp_group=None, keep_last: int = 2):
        self.root = root
        self.model = _unwrap(model)
        self.engine = engine if engine is not None else _engine_of(model)
        self.dp_group = dp_group if dp_group is not None else (self.engine.group if self.engine is not None else None)
        self.keep_last = keep_last

    def _dir(self, step: int) -> str:
        return os.path.join(self.root, f"step{step:08d}")

    def _full_shard(self) -> bool:
        return self.engine is not None and hasattr(self.engine, "full_state_dict")

    def save(self, step: int, extra: Optional[dict] = None):
        rank = _rank()
        d = self._dir(step)
        if rank == 0:
            os.makedirs(d, exist_ok=True)
        _barrier()
        dp_rank = dist.get_rank(self.dp_group) if (dist.is_initialized() and self.dp_group is not None) else \
            (_rank() if self.engine is not None and self.engine.world > 1 else 0)
        # the global rank whose file holds this rank's model-parallel slice: dp-rank 0 of this rank's dp group
        if dist.is_initialized() and self.dp_group is not None:
            model_src = dist.get_global_rank(self.dp_group, 0)
        else:
            model_src = 0 if (self.engine is not None and self.engine.world > 1) else rank
        state = {"step": int(step), "rng": rng_state(), "extra": extra or {}, "model_src": int(model_src)}
        # model shard: data-parallel replicas are identical -> only dp-rank 0 of each model-parallel slice writes
        if self._full_shard():
            # FULL_SHARD: the module's parameters are released between uses; gather the full state (collective)
            sd = self.engine.full_state_dict(rank0_only=True, offload_to_cpu=True)
            if dp_rank == 0:
                state["model"] = sd
        elif dp_rank == 0 or self.engine is None:
            if self.engine is not None:
                self.engine.synchronize()
            state["model"] = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        if self.engine is not None and self.engine.opt_cfg is not None:
            state["optim"] = self.engine.optimizer_state_dict()
        torch.save(state, os.path.join(d, f"rank{rank}.pt.tmp"))
        os.replace(os.path.join(d, f"rank{rank}.pt.tmp"), os.path.join(d, f"rank{rank}.pt"))
        _barrier()
        if rank == 0:
            meta = {"step": step, "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                    "dp_world": self.engine.world if self.engine is not None else 1}
            if self.engine is None:   # without an engine or a dp group every rank holds its own (model-parallel) part
                meta["dp_world"] = dist.get_world_size(self.dp_group) if self.dp_group is not None else 1
            with open(os.path.join(d, "meta.json"), "w") as fh:
                json.dump(meta, fh)
            self._gc()
        _barrier()

    def _gc(self):
        steps = sorted(glob.glob(os.path.join(self.root, "step*")))
        for old in steps[:-self.keep_last] if self.keep_last > 0 else []:
            for f in glob.glob(os.path.join(old, "*")):
                os.remove(f)
            os.rmdir(old)

    def latest(self) -> Optional[str]:
        done = [d for d in sorted(glob.glob(os.path.join(self.root, "step*"))) if os.path.exists(os.path.join(d, "meta.json"))]
        return done[-1] if done else None

    def load(self, path: Optional[str] = None) -> int:
        """Restore from ``path`` (default: latest complete checkpoint). Returns the step (0 if none)."""
        path = path or self.latest()
        if path is None:
            return 0
        meta = json.load(open(os.path.join(path, "meta.json")))
        rank = _rank()
        world = dist.get_world_size() if dist.is_initialized() else 1
        same_world = meta["world_size"] == world
        if not same_world and meta["world_size"] != meta.get("dp_world", meta["world_size"]):
            raise ValueError(f"{path}: saved with model parallelism ({meta['world_size']} ranks, data-parallel "
                             f"{meta['dp_world']}); resuming at another world size ({world}) is only supported for "
                             f"pure data parallelism -- use save_checkpoint / load_checkpoint to change the layout")
        mine = os.path.join(path, f"rank{rank}.pt")
        state = torch.load(mine, map_location="cpu", weights_only=True) if (same_world and os.path.exists(mine)) else {}
        model_sd = state.get("model")
        if model_sd is None:
            # a data-parallel replica that did not write the model: its slice's file (dp-rank 0 of its dp group);
            # pure data parallelism at another world size: rank 0 holds the whole model
            src = int(state.get("model_src", 0))
            model_sd = torch.load(os.path.join(path, f"rank{src}.pt"), map_location="cpu", weights_only=True)["model"]
        if self.engine is not None:
            self.engine.load_full_state_dict(model_sd)
        else:
            self.model.load_state_dict(model_sd)
        if self.engine is not None and self.engine.opt_cfg is not None:
            if same_world and "optim" in state:
                self.engine.load_optimizer_state_dict(state["optim"])
            else:
                shards = [torch.load(f, map_location="cpu", weights_only=True)["optim"]
                          for f in sorted(glob.glob(os.path.join(path, "rank*.pt")),
                                          key=lambda s: int(os.path.basename(s)[4:-3]))]
                reshard_engine_state(self.engine, shards)
        if "rng" in state:
            set_rng_state(state["rng"])
        return int(meta["step"])


@torch.no_grad()
def reshard_engine_state(engine, shards: list[dict]):
    """Rebuild the engine's optimizer state from the per-rank states of a run with another dp world size (and
    possibly another bucket partition, e.g. a different ``bucket_cap_mb`` or the world-dependent 'calibrate' /
    'auto' sizes).

    Every saved rank stored its slice of every group (bucket / unit), each group padded to ALIGN * world.  The
    saved ``group_real`` (unpadded group lengths) gives the OLD partition; stripping each old group's padding yields
    the dense sequence of aligned parameter segments, which is the same for any partition of the same model (the
    parameter order does not depend on where the buckets are cut) and is re-cut into this engine's groups.  A
    checkpoint without ``group_real`` (older format) must match this engine's partition exactly; a mismatch raises
    instead of silently leaving the fp32 master / AdamW moments unrestored.
    """
    old_world, old_sharded = shards[0]["world"], shards[0]["shard"]
    if shards[0].get("kind", "dp") != ("zero3" if hasattr(engine, "full_state_dict") else "dp"):
        raise ValueError("reshard_engine_state: checkpoint written by another engine kind; use the consolidated "
                         "save_checkpoint/load_checkpoint format to change strategy")
    new_real = [sum(align_up(p.numel()) for p in g.params) for g in engine.groups]
    old_real = shards[0].get("group_real")
    if old_real is None:
        old_real = new_real
        old_total = sum(align_up(r, ALIGN * old_world) for r in old_real)
        if "total" in shards[0] and int(shards[0]["total"]) != old_total:
            raise ValueError(f"reshard_engine_state: the checkpoint's bucket partition (total {shards[0]['total']}) "
                             f"differs from this engine's ({old_total}) and the checkpoint records no group sizes; "
                             f"resume with the original bucket partition")
    if sum(old_real) != sum(new_real):
        raise ValueError(f"reshard_engine_state: checkpoint holds {sum(old_real)} parameter elements, this engine "
                         f"{sum(new_real)} (another model?)")
    sizes = [align_up(r, ALIGN * old_world) for r in old_real]
    old_total = sum(sizes)

    def assemble(get):
        """Dense (padding-free) concatenation of the old groups' real parts."""
        if not old_sharded:
            full = get(shards[0])
        else:
            parts, offs = [], [0] * old_world
            for sz in sizes:
                sh = sz // old_world
                for r in range(old_world):
                    parts.append(get(shards[r])[offs[r]:offs[r] + sh])
                    offs[r] += sh
            full = torch.cat(parts)
        if full.numel() != old_total:
            raise ValueError(f"reshard_engine_state: saved vector of {full.numel()} elements, layout needs {old_total}")
        dense, o = [], 0
        for sz, real in zip(sizes, old_real):
            dense.append(full[o:o + real])
            o += sz
        return torch.cat(dense)

    n_state = len(shards[0]["state"])
    dsts = [engine.master] + list(engine.opt_state)
    if n_state != len(engine.opt_state):
        raise ValueError(f"reshard_engine_state: {n_state} optimizer-state vectors saved, engine has "
                         f"{len(engine.opt_state)} (another optimizer?)")
    getters = [lambda s: s["master"]] + [lambda s, i=i: s["state"][i] for i in range(n_state)]
    # The caller loaded the checkpoint's model first, so the engine's master currently holds those weights (rounded
    # to the parameter dtype).  The re-cut fp32 master must round to exactly them: a wrong partition guess (older
    # checkpoints without group sizes) shows up here instead of training on scrambled optimizer state.
    current = engine.master.detach().cpu().clone()
    pdt = getattr(engine, "param_dtype", torch.float32)
    for k, (get, dst) in enumerate(zip(getters, dsts)):
        if dst.numel() == 1 and get(shards[0]).numel() == 1:
            continue   # SGD without momentum: a one-element dummy, not laid out like the master
        dense = assemble(get)
        o = 0
        for g, real in zip(engine.groups, new_real):
            t = torch.zeros(g.numel, dtype=torch.float32)
            t[:real] = dense[o:o + real]
            mine = t[_rank_slice(engine, g)]
            if k == 0 and not torch.equal(mine.to(pdt).float(), current[engine.opt_slice(g)]):
                raise ValueError("reshard_engine_state: the checkpoint's fp32 master does not match its model weights "
                                 "under this engine's bucket partition (saved with another bucket_cap_mb and no "
                                 "recorded group sizes?); resume with the original bucket partition")
            dst[engine.opt_slice(g)].copy_(mine)
            o += real
    engine.step_count = int(shards[0]["step"])
    engine.refresh_params_from_master()
