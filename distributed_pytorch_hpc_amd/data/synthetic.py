"""Synthetic datasets and on-device batch generators.

Capability parity with the reference's datasets: ``MyTrainDataset`` (2000 x (rand(20), rand(1)),
multinode_ddp_basic.py:89-105), ``SimpleDataset`` (randn features + binary labels, distributed_dataloader.py:143-156),
``ERA5Dataset`` (random [C, lat, lon] fields, multinode_ddp_unet.py:145-164), synthetic tokens and synthetic
images (scripts/main.py:268-271).  The reference draws a fresh randn(65,181,360) per sample in CPU loader workers,
which makes its UNet driver loader-bound (X16); ``DeviceBatches`` generates whole batches on the GPU instead,
deterministically per (seed, rank, step), with zero host traffic.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class MyTrainDataset(Dataset):
    def __init__(self, size: int = 2000, in_features: int = 20, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.data = [(torch.rand(in_features, generator=g), torch.rand(1, generator=g)) for _ in range(size)]

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        return self.data[i]


class SimpleDataset(Dataset):
    def __init__(self, size: int = 1000, input_dim: int = 10, num_classes: int = 2, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(size, input_dim, generator=g)
        self.y = torch.randint(0, num_classes, (size,), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]


class ERA5Dataset(Dataset):
    """Random ERA5-shaped (input, target) pairs; deterministic per index (seeded generator per item)."""

    def __init__(self, num_samples: int = 64, channels: int = 65, lat: int = 181, lon: int = 360, seed: int = 0):
        self.n, self.shape, self.seed = num_samples, (channels, lat, lon), seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randn(self.shape, generator=g), torch.randn(self.shape, generator=g)


class TokenDataset(Dataset):
    """Random token sequences of length seq_len + 1 (inputs = [:-1], targets = [1:])."""

    def __init__(self, num_samples: int, seq_len: int, vocab_size: int, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.data = torch.randint(0, vocab_size, (num_samples, seq_len + 1), generator=g)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        t = self.data[i]
        return t[:-1], t[1:]


class DeviceBatches:
    """Infinite on-device synthetic batches: kind in {"tokens", "images", "era5", "regression"}."""

    def __init__(self, kind: str, batch_size: int, device, seed: int = 0, rank: int = 0, *, seq_len: int = 256,
                 vocab_size: int = 32000, image_size: int = 224, num_classes: int = 1000, channels: int = 65,
                 lat: int = 181, lon: int = 360, dtype=torch.float32, fixed: bool = False):
        self.kind, self.b, self.device, self.dtype = kind, batch_size, torch.device(device), dtype
        self.seq_len, self.vocab, self.img, self.ncls = seq_len, vocab_size, image_size, num_classes
        self.c, self.lat, self.lon = channels, lat, lon
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 7919 + rank)
        self.fixed = fixed
        self._cache = None

    def __iter__(self):
        return self

    def __next__(self):
        if self.fixed and self._cache is not None:
            return self._cache
        g, d = self.gen, self.device
        if self.kind == "tokens":
            t = torch.randint(0, self.vocab, (self.b, self.seq_len + 1), device=d, generator=g)
            out = (t[:, :-1], t[:, 1:])
        elif self.kind == "images":
            x = torch.rand(self.b, 3, self.img, self.img, device=d, generator=g, dtype=self.dtype)
            out = (x, torch.randint(0, self.ncls, (self.b,), device=d, generator=g))
        elif self.kind == "era5":
            shp = (self.b, self.c, self.lat, self.lon)
            out = (torch.randn(shp, device=d, generator=g, dtype=self.dtype),
                   torch.randn(shp, device=d, generator=g, dtype=self.dtype))
        elif self.kind == "regression":
            out = (torch.rand(self.b, 20, device=d, generator=g), torch.rand(self.b, 1, device=d, generator=g))
        else:
            raise ValueError(self.kind)
        if self.fixed:
            self._cache = out
        return out
