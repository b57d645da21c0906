"""Generic epoch-based training loop shared by every data-parallel example driver.

Reference capability: the ``Trainer`` of scripts/01_data_parallel_ddp/multinode_ddp_basic.py:114-208
(``_run_batch / _run_epoch / _save_snapshot / _load_snapshot / train`` with per-epoch timing and a resumable
``snapshot.pt``), the throughput loops of multinode_ddp_unet.py:318-398 (global samples/s per batch / epoch /
run), resnet_fsdp_training.py:90-155 (``train_epoch`` + ``test`` with loss/accuracy) and scripts/main.py:332-376
(average epoch time excluding epoch 0).

Differences by design:
  * one checkpoint path for every layout: consolidated ``save_checkpoint`` for replicated optimizers, the
    ``ShardedCheckpointer`` when the optimizer state is sharded (FSDP / ZeRO engines) -- reference defect X15;
  * evaluation is collective (every rank evaluates its shard, sums are all-reduced), so it also works under
    FSDP -- reference defect X9 (rank-0-only eval hangs with FSDP);
  * throughput is measured with device-synchronised timers and reported as GLOBAL samples/s (x world).
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..utils import checkpointing as ckpt
from ..utils.logging import get_logger
from ..utils.metrics import MetricsLogger, sync

log = get_logger("dph.trainer")


def _batch_size(x) -> int:
    if torch.is_tensor(x):
        return x.shape[0]
    if isinstance(x, (list, tuple)) and x:
        return _batch_size(x[0])
    return 1


def _to(x, device):
    if torch.is_tensor(x):
        return x.to(device, non_blocking=True)
    if isinstance(x, (list, tuple)):
        return type(x)(_to(t, device) for t in x)
    return x


@dataclass
class EpochStats:
    epoch: int
    loss: float
    seconds: float
    samples: int
    samples_per_sec: float   # global (all data-parallel ranks)
    extra: dict = field(default_factory=dict)


class Trainer:
    """Epoch loop over a (sharded) DataLoader.

    ``model`` may be a plain module, ``DDP`` / ``FSDP`` wrapper or any callable module; ``optimizer`` a
    ``torch.optim`` optimizer or the engine facade returned by ``DDP.make_optimizer`` / ``FSDP.make_optimizer``.
    ``dp_world`` is the number of data-parallel replicas used for global throughput (defaults to the world size).
    """

    def __init__(self, model, optimizer, train_loader, loss_fn: Callable, device, *,
                 sampler=None, snapshot_path: Optional[str] = None, save_every: int = 0, log_every: int = 10,
                 max_steps_per_epoch: Optional[int] = None, dp_world: Optional[int] = None,
                 autocast_dtype: Optional[torch.dtype] = None, grad_clip: Optional[float] = None,
                 scheduler=None, metrics_file: Optional[str] = None, profiler=None, cuda_graph: bool = False,
                 graph_warmup: int = 3):
        self.model = model
        self.optimizer = optimizer
        self.loader = train_loader
        self.loss_fn = loss_fn
        self.device = torch.device(device)
        self.sampler = sampler
        self.snapshot_path = snapshot_path
        self.save_every = save_every
        self.log_every = log_every
        self.max_steps = max_steps_per_epoch
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.dp_world = dp_world or self.world
        self.autocast_dtype = autocast_dtype
        self.grad_clip = grad_clip
        self.scheduler = scheduler
        self.metrics = MetricsLogger(metrics_file, self.rank)
        self.profiler = profiler
        # whole-step HIP graph (runtime/graphs.py): eager for `graph_warmup` steps, then capture + replay
        self.cuda_graph = bool(cuda_graph) and self.device.type == "cuda"
        self.graph_warmup = graph_warmup
        self._graphed = None
        self.epochs_run = 0
        self.global_step = 0
        self.history: list[EpochStats] = []
        self.engine = getattr(optimizer, "engine", None)
        # sharded optimizer state (ZeRO-2 / FULL_SHARD): per-rank snapshot files instead of one consolidated file
        self._sharded = bool(self.engine is not None and getattr(self.engine, "sharded_state", False))
        if snapshot_path:
            self._load_snapshot()

    # ------------------------------------------------------------------------------------------ snapshots
    def _checkpointer(self):
        return ckpt.ShardedCheckpointer(self.snapshot_path, self.model, engine=self.engine, keep_last=1)

    def _save_snapshot(self, epoch: int):
        if self.engine is not None:
            self.engine.synchronize()
        if self._sharded:
            self._checkpointer().save(epoch, extra={"epochs_run": epoch})
        else:
            ckpt.save_checkpoint(self.model, self.optimizer, epoch, self.snapshot_path,
                                 extra={"global_step": self.global_step})
        if self.rank == 0:
            log.info("epoch %d | snapshot saved at %s", epoch, self.snapshot_path)

    def _load_snapshot(self):
        if self._sharded:
            step = self._checkpointer().load()
        else:
            step = ckpt.load_checkpoint(self.model, self.optimizer, self.snapshot_path, device=self.device)
        if step:
            self.epochs_run = step
            if self.rank == 0:
                log.info("resuming training from snapshot at epoch %d", step)

    # ------------------------------------------------------------------------------------------ steps
    def _autocast(self):
        if self.autocast_dtype is None:
            return contextlib.nullcontext()
        # a captured step must not keep autocast's per-step weight-cast cache (it would pin the capture's copies)
        return torch.autocast(device_type=self.device.type, dtype=self.autocast_dtype,
                              cache_enabled=not self.cuda_graph)

    def _step_body(self, source, targets) -> torch.Tensor:
        self.optimizer.zero_grad(set_to_none=True)
        with self._autocast():
            output = self.model(source)
            loss = self.loss_fn(output, targets)
        loss.backward()
        if self.grad_clip is not None and self.engine is None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip)
        self.optimizer.step()
        return loss.detach()

    def _run_batch(self, source, targets) -> torch.Tensor:
        if self.cuda_graph and torch.is_tensor(source) and torch.is_tensor(targets):
            if self._graphed is None:
                from ..runtime.graphs import GraphedStep

                self._graphed = GraphedStep(self._step_body, optimizer=self.optimizer, warmup=self.graph_warmup)
            lr = self.optimizer.param_groups[0]["lr"] if hasattr(self.optimizer, "param_groups") else None
            loss = self._graphed(source, targets, lr=lr if isinstance(lr, float) else None)
        else:
            loss = self._step_body(source, targets)
        if self.scheduler is not None:
            self.scheduler.step()
        self.global_step += 1
        return loss

    def _run_epoch(self, epoch: int) -> EpochStats:
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)
        if hasattr(self.model, "train"):
            self.model.train()
        sync()
        t0 = time.perf_counter()
        tb = t0
        loss_sum = torch.zeros((), device=self.device)
        n_batches = samples = 0
        for i, (source, targets) in enumerate(self.loader):
            if self.max_steps is not None and i >= self.max_steps:
                break
            source, targets = _to(source, self.device), _to(targets, self.device)
            loss = self._run_batch(source, targets)
            loss_sum += loss.float()
            n_batches += 1
            bs = _batch_size(source)
            samples += bs
            if self.profiler is not None:
                self.profiler.step()
            if self.log_every and (i + 1) % self.log_every == 0:
                sync()
                now = time.perf_counter()
                sps = self.log_every * bs * self.dp_world / (now - tb)
                tb = now
                if self.rank == 0:
                    log.info("epoch %d | batch %d | loss %.5f | %.1f samples/s (global)", epoch, i + 1,
                             loss.item(), sps)
                self.metrics.log(self.global_step, epoch=epoch, loss=loss.item(), samples_per_sec=sps)
        if self.engine is not None:
            self.engine.synchronize()
        sync()
        dt = time.perf_counter() - t0
        mean_loss = (loss_sum / max(n_batches, 1)).item()
        st = EpochStats(epoch, mean_loss, dt, samples * self.dp_world, samples * self.dp_world / max(dt, 1e-9))
        if self.rank == 0:
            log.info("epoch %d done | %d steps | loss %.5f | %.2f s | %.1f samples/s (global)", epoch, n_batches,
                     mean_loss, dt, st.samples_per_sec)
        self.metrics.log(self.global_step, epoch=epoch, epoch_loss=mean_loss, epoch_seconds=dt,
                         epoch_samples_per_sec=st.samples_per_sec)
        return st

    def train(self, max_epochs: int) -> dict:
        for epoch in range(self.epochs_run, max_epochs):
            st = self._run_epoch(epoch)
            self.history.append(st)
            self.epochs_run = epoch + 1
            if self.snapshot_path and self.save_every and (epoch + 1) % self.save_every == 0:
                self._save_snapshot(epoch + 1)
        return self.summary()

    def summary(self) -> dict:
        times = [h.seconds for h in self.history]
        steady = times[1:] if len(times) > 1 else times
        out = {
            "epochs": len(times),
            "total_seconds": sum(times),
            "avg_epoch_seconds": sum(times) / max(len(times), 1),
            "avg_epoch_seconds_excl_first": sum(steady) / max(len(steady), 1),
            "samples_per_sec": (sum(h.samples for h in self.history) / max(sum(times), 1e-9)),
            "samples_per_sec_per_gpu": (sum(h.samples for h in self.history) / max(sum(times), 1e-9)) / self.dp_world,
            # steady state: epochs after the first (kernel autotuning / allocator warm-up land in epoch 0)
            "samples_per_sec_excl_first": (sum(h.samples for h in self.history[1:]) / max(sum(steady), 1e-9)
                                           if len(self.history) > 1 else None),
            "final_loss": self.history[-1].loss if self.history else None,
        }
        if self.rank == 0 and self.history:
            log.info("training summary: %s", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()})
        return out

    # ------------------------------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, loader, max_steps: Optional[int] = None) -> dict:
        """Collective evaluation: every rank scores its shard; loss sum / correct / count are all-reduced."""
        if hasattr(self.model, "eval"):
            self.model.eval()
        tot = torch.zeros(3, dtype=torch.float64, device=self.device)   # loss_sum, correct, count
        for i, (source, targets) in enumerate(loader):
            if max_steps is not None and i >= max_steps:
                break
            source, targets = _to(source, self.device), _to(targets, self.device)
            with self._autocast():
                out = self.model(source)
                loss = self.loss_fn(out, targets)
            n = _batch_size(source)
            tot[0] += loss.double() * n
            tot[2] += n
            if out.dim() == 2 and targets.dim() == 1 and not targets.is_floating_point():
                tot[1] += (out.argmax(1) == targets).sum()
        if dist.is_initialized():
            dist.all_reduce(tot)
        if hasattr(self.model, "train"):
            self.model.train()
        cnt = max(tot[2].item(), 1.0)
        return {"loss": tot[0].item() / cnt, "accuracy": tot[1].item() / cnt, "samples": int(tot[2].item())}


def _share_cpu_threads(info):
    """CPU ranks of one node split the cores instead of each starting one intra-op thread per core: with 2 ranks on
    8 cores the oversubscribed default ran ResNet-50 DDP/gloo at 3.4 img/s, 4 threads per rank at 16.8.  An explicit
    OMP_NUM_THREADS wins."""
    if os.environ.get("OMP_NUM_THREADS"):
        return
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0) or (info.world_size if info.world_size > 1 else 1)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:   # non-Linux
        cores = os.cpu_count() or 1
    torch.set_num_threads(max(1, cores // max(local_world, 1)))


def setup_run(backend: Optional[str] = None, device: Optional[str] = None, seed: int = 0, verbose: bool = True):
    """(rank, world, local, device) for any launcher; CPU+gloo when ``device == 'cpu'`` or no GPU is present."""
    from ..runtime import env as rt

    if device == "cpu" or not torch.cuda.is_available():
        backend = "gloo"
    info = rt.get_rank_info()
    if info.world_size > 1:
        rank, world, local = rt.init_distributed(backend=backend, verbose=verbose)
    else:
        rank, world, local = 0, 1, 0
    if device == "cpu" or not torch.cuda.is_available() or backend == "gloo":
        dev = torch.device("cpu")
        _share_cpu_threads(info)
    else:
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(seed)
    return rank, world, local, dev
