"""Training metrics: throughput, MFU, HBM peak, scaling efficiency, JSONL sink.

The reference only prints samples/s / tokens/s / epoch times (scripts/01_data_parallel_ddp/multinode_ddp_unet.py:351-398,
scripts/04_pipeline_parallel_pp/03_pipeline_training.py:282-289, scripts/main.py:376-397).  ``StepTimer`` uses
device-synchronised wall time, ``MetricsLogger`` writes one JSON line per logged step from rank 0 (and a
per-rank summary on request), ``scaling_efficiency`` = T1 * N / TN for weak-scaling throughput curves.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import torch

MI355X_BF16_DENSE_FLOPS = 2.5e15


def sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


class StepTimer:
    def __init__(self, skip_first: int = 0):
        self.skip_first = skip_first
        self.times: list[float] = []
        self._t0: Optional[float] = None
        self._n = 0

    def start(self):
        sync()
        self._t0 = time.perf_counter()

    def stop(self) -> float:
        sync()
        dt = time.perf_counter() - self._t0
        self._n += 1
        if self._n > self.skip_first:
            self.times.append(dt)
        return dt

    @property
    def mean(self) -> float:
        return sum(self.times) / max(len(self.times), 1)


def mfu(tokens_per_sec_per_gpu: float, flops_per_token: float, peak: float = MI355X_BF16_DENSE_FLOPS) -> float:
    return tokens_per_sec_per_gpu * flops_per_token / peak


def scaling_efficiency(throughput: dict[int, float], weak: bool = True) -> dict[int, float]:
    """{N: efficiency}: weak scaling -> X_N / (N * X_1); strong -> T_1 / (N * T_N) expressed on throughput too."""
    base = throughput[min(throughput)]
    n0 = min(throughput)
    return {n: (x / base) / (n / n0) for n, x in sorted(throughput.items())}


def peak_hbm_gb() -> float:
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        return torch.cuda.max_memory_allocated() / 1e9
    return 0.0


class MetricsLogger:
    def __init__(self, path: Optional[str] = None, rank: Optional[int] = None):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.path = path
        self._fh = open(path, "a", buffering=1) if (path and self.rank == 0) else None

    def log(self, step: int, **kv):
        rec = {"step": step, "time": time.time(), **{k: (float(v) if torch.is_tensor(v) else v) for k, v in kv.items()}}
        if self._fh:
            self._fh.write(json.dumps(rec) + "\n")
        return rec

    def close(self):
        if self._fh:
            self._fh.close()
