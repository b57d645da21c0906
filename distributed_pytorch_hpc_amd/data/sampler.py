"""Data-parallel-rank-aware distributed sampling.

The reference shards data by WORLD rank even inside a TP mesh, so tensor-parallel peers see different inputs
(scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:303-305, defect X6).  ``DistributedSampler`` here takes the
data-parallel coordinates explicitly (``num_replicas = dp size``, ``rank = dp rank``), so TP/PP/CP peers of
one replica read identical samples.  Same epoch-seeded shuffling / padding semantics as
torch.utils.data.DistributedSampler (``set_epoch`` each epoch).
"""
from __future__ import annotations

import math

import torch
from torch.utils.data import DataLoader, Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.dataset, self.num_replicas, self.rank = dataset, num_replicas, rank
        self.shuffle, self.seed, self.drop_last, self.epoch = shuffle, seed, drop_last, 0
        n = len(dataset)
        if drop_last and n % num_replicas:
            self.num_samples = n // num_replicas
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __iter__(self):
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g).tolist()
        else:
            idx = list(range(n))
        if self.drop_last:
            idx = idx[: self.total_size]
        else:
            pad = self.total_size - len(idx)
            idx = idx + (idx * math.ceil(max(pad, 1) / max(len(idx), 1)))[:pad]
        return iter(idx[self.rank: self.total_size: self.num_replicas])

    def __len__(self):
        return self.num_samples


def dp_dataloader(dataset, batch_size: int, dp_size: int = 1, dp_rank: int = 0, shuffle: bool = True, seed: int = 0,
                  num_workers: int = 2, pin_memory: bool = True, drop_last: bool = False):
    sampler = DistributedSampler(dataset, dp_size, dp_rank, shuffle, seed, drop_last)
    return DataLoader(dataset, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                      pin_memory=pin_memory and torch.cuda.is_available(), drop_last=drop_last,
                      persistent_workers=num_workers > 0), sampler
