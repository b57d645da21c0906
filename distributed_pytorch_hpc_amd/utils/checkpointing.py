"""Checkpoint / resume for every parallel layout of the framework.

Reference capability: utils/checkpointing.py:23-88 (rank-0 save of model+optimizer+epoch, barrier, load with
map_location), the DDP ``snapshot.pt`` auto-resume (scripts/01_data_parallel_ddp/multinode_ddp_basic.py:144-196)
and the FSDP FULL_STATE_DICT rank-0 consolidation (scripts/02_fully_sharded_fsdp/multinode_fsdp_unet.py:282-298).
Fixes the reference defects X15 (one module used everywhere; a single writer per job, not per node).

Two formats:
  * ``save_checkpoint`` / ``load_checkpoint``: consolidated single file written by global rank 0 (small models,
    interoperability).  Model state is unwrapped from ``.module``.
  * ``ShardedCheckpointer``: one directory per step, ``rank{r}.pt`` per rank holding that rank's model shard
    (TP/PP shards; data-parallel replicas are written by their dp-rank-0 only) and optimizer shard (the
    DataParallelEngine's fp32 master / m / v slice) + ``meta.json``.  Loading at a DIFFERENT data-parallel world
    size re-slices the engine's flat optimizer state (``reshard_engine_state``).
Both store the step/epoch, torch + HIP RNG state and arbitrary extra metadata; files are loaded with
``weights_only=True`` (tensors, numbers, strings, lists, dicts only).
"""
from __future__ import annotations

import glob
import json
import os
from typing import Optional

import torch
import torch.distributed as dist


def _rank():
    return dist.get_rank() if dist.is_initialized() else 0


def _barrier():
    if dist.is_initialized():
        dist.barrier()


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


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


def save_checkpoint(model, optimizer, epoch: int, path: str, extra: Optional[dict] = None, rank: Optional[int] = None):
    """Consolidated checkpoint from global rank 0; every rank must call it (barrier)."""
    rank = _rank() if rank is None else rank
    if rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        state = {"model_state_dict": {k: v.detach().cpu() for k, v in _unwrap(model).state_dict().items()},
                 "optimizer_state_dict": optimizer.state_dict() if optimizer is not None else None,
                 "epoch": int(epoch), "rng": rng_state(), "extra": extra or {}}
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)   # atomic: a crash never leaves a truncated checkpoint
    _barrier()


def load_checkpoint(model, optimizer, path: str, device=None) -> int:
    """Restores model (+optimizer) in place; returns the stored epoch, or 0 when ``path`` is missing."""
    if not os.path.exists(path):
        return 0
    state = torch.load(path, map_location=device or "cpu", weights_only=True)
    _unwrap(model).load_state_dict(state["model_state_dict"])
    if optimizer is not None and state.get("optimizer_state_dict") is not None:
        optimizer.load_state_dict(state["optimizer_state_dict"])
    if "rng" in state:
        set_rng_state(state["rng"])
    return int(state.get("epoch", 0))


# ------------------------------------------------------------------------------------------------ sharded
class ShardedCheckpointer:
    def __init__(self, root: str, model, engine=None, dp_group=None, keep_last: int = 2):
        self.root = root
        self.model = _unwrap(model)
        self.engine = engine
        self.dp_group = dp_group if dp_group is not None else (engine.group if engine is not None else None)
        self.keep_last = keep_last

    def _dir(self, step: int) -> str:
        return os.path.join(self.root, f"step{step:08d}")

    def save(self, step: int, extra: Optional[dict] = None):
        rank = _rank()
        d = self._dir(step)
        if rank == 0:
            os.makedirs(d, exist_ok=True)
        _barrier()
        dp_rank = dist.get_rank(self.dp_group) if (dist.is_initialized() and self.dp_group is not None) else \
            (_rank() if self.engine is not None and self.engine.world > 1 else 0)
        state = {"step": int(step), "rng": rng_state(), "extra": extra or {}}
        # model shard: data-parallel replicas are identical -> only dp-rank 0 of each model-parallel slice writes
        if dp_rank == 0 or self.engine is None:
            state["model"] = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        if self.engine is not None and self.engine.opt_cfg is not None:
            state["optim"] = self.engine.optimizer_state_dict()
        torch.save(state, os.path.join(d, f"rank{rank}.pt.tmp"))
        os.replace(os.path.join(d, f"rank{rank}.pt.tmp"), os.path.join(d, f"rank{rank}.pt"))
        _barrier()
        if rank == 0:
            meta = {"step": step, "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                    "dp_world": self.engine.world if self.engine is not None else 1}
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
        mine = os.path.join(path, f"rank{rank}.pt")
        state = torch.load(mine, map_location="cpu", weights_only=True) if (same_world and os.path.exists(mine)) else {}
        model_sd = state.get("model")
        if model_sd is None:   # a dp replica that did not write the model: read rank 0 of the same slice (rank 0)
            model_sd = torch.load(os.path.join(path, "rank0.pt"), map_location="cpu", weights_only=True)["model"]
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


def reshard_engine_state(engine, shards: list[dict]):
    """Rebuild the engine's optimizer state from the per-rank states of a run with another dp world size.

    Every saved rank stored its slice of every bucket (bucket layout is a pure function of the model and the
    world size); the full flat fp32 vectors are reassembled from the OLD layout, then re-sliced for this engine.
    """
    from ..parallel.data_parallel import DataParallelEngine  # noqa: F401  (type reference)

    old_world = shards[0]["world"]
    old_sharded = shards[0]["shard"]
    if not old_sharded:
        full = {"master": shards[0]["master"], "state": shards[0]["state"]}
    else:
        # old bucket sizes: recompute from this engine's parameter order with the old world's padding
        from ..utils.flat import ALIGN, align_up

        sizes = []
        for b in engine.buckets:
            n = sum(align_up(p.numel()) for p in b.params)
            sizes.append(align_up(n, ALIGN * old_world))
        def assemble(key, idx=None):
            parts = []
            offs = [0] * old_world
            for sz in sizes:
                sh = sz // old_world
                for r in range(old_world):
                    src = shards[r][key] if idx is None else shards[r][key][idx]
                    parts.append(src[offs[r]:offs[r] + sh])
                    offs[r] += sh
            return torch.cat(parts)
        full = {"master": assemble("master"), "state": [assemble("state", i) for i in range(len(shards[0]["state"]))]}
    # full vectors are in the old padded layout; re-slice per bucket into the new layout
    from ..utils.flat import ALIGN, align_up

    def old_bucket_offsets(world):
        offs, o = [], 0
        for b in engine.buckets:
            n = align_up(sum(align_up(p.numel()) for p in b.params), ALIGN * world)
            offs.append((o, n))
            o += n
        return offs

    old = old_bucket_offsets(old_world if old_sharded else engine.world)
    if not old_sharded:
        old = old_bucket_offsets(old_world)
    with torch.no_grad():
        for b, (o, n) in zip(engine.buckets, old):
            real = sum(align_up(p.numel()) for p in b.params)
            src_m = full["master"][o:o + real]
            dst = torch.zeros(b.numel, dtype=torch.float32)
            dst[:real] = src_m
            engine_slice = slice(b.offset, b.offset + b.numel)
            if engine.shard:
                s = engine.rank * b.shard_numel
                engine.master_view(b).copy_(dst[s:s + b.shard_numel])
                for i, st in enumerate(engine.opt_state):
                    t = torch.zeros(b.numel, dtype=torch.float32)
                    t[:real] = full["state"][i][o:o + real]
                    st[b.shard_offset:b.shard_offset + b.shard_numel].copy_(t[s:s + b.shard_numel])
            else:
                engine.master[engine_slice].copy_(dst)
                for i, st in enumerate(engine.opt_state):
                    t = torch.zeros(b.numel, dtype=torch.float32)
                    t[:real] = full["state"][i][o:o + real]
                    st[engine_slice].copy_(t)
            engine.param_shard_view(b).copy_(engine.master_view(b))
    engine.step_count = int(shards[0]["step"])
    if engine.shard:
        for b in engine.buckets:
            dist.all_gather_into_tensor(engine.param_view(b), engine.param_shard_view(b).clone(), group=engine.group)
