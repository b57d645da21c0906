"""CIFAR-10 for the ResNet walkthroughs, with the whole dataset resident in HBM and batches assembled on the GPU.

Reference capability (SURVEY.md D-cifar): scripts/02_fully_sharded_fsdp/resnet_fsdp_training.py:45-87 (torchvision
``CIFAR10(download=True)`` on rank 0 + barrier, train transform RandomCrop(32, padding=4) + RandomHorizontalFlip +
ToTensor + Normalize, ``DistributedSampler`` + ``set_epoch``) and scripts/main.py:274-306.  torchvision and the network
are unavailable here, and the reference's pickled ``cifar-10-batches-py`` would need unpickling, so this reads the
binary distribution instead (``cifar-10-batches-bin``: ``data_batch_{1..5}.bin`` / ``test_batch.bin``, records of one
label byte + 3072 pixel bytes in CHW order) straight into numpy -- nothing is executed from the files.

MI355X-first loader: 60,000 images are 184 MB of uint8, so the split is copied to the device ONCE and every batch
is one gather + augment kernel (csrc/imageaug.hip ``image_augment``) reading it -- no DataLoader workers, no host
decode, no pinned-memory copies per step.  Crop offsets and flips are drawn on the device from a seeded generator;
sampling is data-parallel-rank aware with the same epoch-seeded permutation / padding rules as ``DistributedSampler``.

    ds = CIFAR10("/data/cifar-10-batches-bin", train=True)
    loader = CIFARDeviceLoader(ds, batch_size=128, device=dev, dp_rank=r, dp_size=w, augment=True, dtype=torch.bfloat16)
    for epoch ...: loader.set_epoch(epoch); for x, y in loader: ...
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

from ..ops import _lib

MEAN = (0.4914, 0.4822, 0.4465)   # the reference's Normalize constants (resnet_fsdp_training.py:51-52, main.py:279-281)
STD = (0.2023, 0.1994, 0.2010)
_REC = 1 + 3 * 32 * 32


def _read_batches(paths: list[str]) -> tuple[np.ndarray, np.ndarray]:
    chunks = []
    for p in paths:
        raw = np.fromfile(p, dtype=np.uint8)
        if raw.size % _REC:
            raise ValueError(f"{p}: {raw.size} bytes is not a whole number of CIFAR-10 records ({_REC} B)")
        chunks.append(raw.reshape(-1, _REC))
    rec = np.concatenate(chunks)
    labels = rec[:, 0].astype(np.int64)
    images = rec[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)   # CHW -> HWC
    return np.ascontiguousarray(images), labels


def write_cifar_bin(path: str, images: np.ndarray, labels: np.ndarray):
    """Write uint8 HWC images [N, 32, 32, 3] + labels in the CIFAR-10 binary record format (tests / conversion)."""
    rec = np.empty((len(labels), _REC), dtype=np.uint8)
    rec[:, 0] = labels
    rec[:, 1:] = images.transpose(0, 3, 1, 2).reshape(len(labels), -1)
    rec.tofile(path)


class CIFAR10(torch.utils.data.Dataset):
    """CIFAR-10 (binary distribution) as uint8 HWC images + int64 labels; ``__getitem__`` gives untransformed
    samples (CPU DataLoader use); ``CIFARDeviceLoader`` is the fast path."""

    def __init__(self, root: str, train: bool = True):
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        paths = [os.path.join(root, n) for n in names]
        missing = [p for p in paths if not os.path.exists(p)]
        if missing:
            raise FileNotFoundError(f"CIFAR-10 binary files not found: {missing} (expected the cifar-10-batches-bin "
                                    f"layout; no download is attempted)")
        self.images, self.labels = _read_batches(paths)
        self.train = train

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        return torch.from_numpy(self.images[i]), int(self.labels[i])


def augment_reference(images_u8: torch.Tensor, params: Optional[torch.Tensor], mean, std, pad: int = 4,
                      channels_last: bool = False, dtype=torch.float32) -> torch.Tensor:
    """Eager reference of the kernel on uint8 HWC images [B, H, W, C] (CPU path and the GPU test oracle)."""
    b, h, w, c = images_u8.shape
    x = images_u8.permute(0, 3, 1, 2).float() / 255.0
    if params is not None:
        x = torch.nn.functional.pad(x, (pad, pad, pad, pad))
        out = torch.empty((b, c, h, w), dtype=torch.float32, device=x.device)
        for i in range(b):
            dy, dx, flip = (int(v) for v in params[i].tolist())
            crop = x[i, :, dy:dy + h, dx:dx + w]
            out[i] = crop.flip(-1) if flip else crop
        x = out
    m = torch.tensor(mean, dtype=torch.float32, device=x.device).view(1, c, 1, 1)
    s = torch.tensor(std, dtype=torch.float32, device=x.device).view(1, c, 1, 1)
    x = ((x - m) * (1.0 / s)).to(dtype)
    return x.contiguous(memory_format=torch.channels_last) if channels_last else x


class CIFARDeviceLoader:
    """Data-parallel batches of a ``CIFAR10`` split assembled on ``device`` (see module docstring).

    One epoch = ``len(self)`` batches of this rank's shard (``drop_last``: full batches only, like the reference's
    training loop; otherwise the last batch is short).  Yields ``(images [B, 3, 32, 32], labels [B])``."""

    def __init__(self, ds: CIFAR10, batch_size: int, device, dp_rank: int = 0, dp_size: int = 1,
                 augment: bool = True, shuffle: bool = True, seed: int = 0, dtype=torch.float32,
                 channels_last: bool = False, drop_last: bool = True, pad: int = 4, mean=MEAN, std=STD):
        self.device = torch.device(device)
        self.images = torch.from_numpy(ds.images).to(self.device)
        self.labels = torch.from_numpy(ds.labels).to(self.device)
        self.b, self.rank, self.world = batch_size, dp_rank, dp_size
        self.augment, self.shuffle, self.seed, self.dtype = augment, shuffle, seed, dtype
        self.channels_last, self.drop_last, self.pad = channels_last, drop_last, pad
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.inv_std = 1.0 / torch.tensor(std, dtype=torch.float32, device=self.device)
        self._mean_t, self._std_t = tuple(mean), tuple(std)
        n = len(ds)
        self.num_samples = math.ceil(n / dp_size)          # DistributedSampler padding rule
        self.total = self.num_samples * dp_size
        self.epoch = 0
        self._gen = torch.Generator(device=self.device)
        self._native = self.device.type == "cuda" and _lib.use_native(self.images)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __len__(self):
        return self.num_samples // self.b if self.drop_last else math.ceil(self.num_samples / self.b)

    def _indices(self) -> torch.Tensor:
        n = len(self.labels)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if self.total > n:
            idx = torch.cat([idx, idx[: self.total - n]])
        return idx[self.rank:self.total:self.world].to(self.device)

    def batch(self, idx: torch.Tensor):
        """Assemble the batch of dataset indices ``idx`` (device int64 [B])."""
        params = None
        if self.augment:
            b = idx.numel()
            off = torch.randint(0, 2 * self.pad + 1, (b, 2), device=self.device, generator=self._gen,
                                dtype=torch.int32)
            flip = torch.randint(0, 2, (b, 1), device=self.device, generator=self._gen, dtype=torch.int32)
            params = torch.cat([off, flip], 1).contiguous()
        if self._native:
            x = _lib.ops().image_augment(self.images, idx, params, self.mean, self.inv_std,
                                         self.pad, self.channels_last, self.dtype == torch.bfloat16)
            if self.dtype not in (torch.float32, torch.bfloat16):
                x = x.to(self.dtype)
        else:
            x = augment_reference(self.images[idx], params, self._mean_t, self._std_t, self.pad, self.channels_last,
                                  self.dtype)
        return x, self.labels[idx]

    def __iter__(self):
        self._gen.manual_seed(self.seed * 1_000_003 + self.epoch * 7919 + self.rank)
        idx = self._indices()
        for i in range(len(self)):
            yield self.batch(idx[i * self.b:(i + 1) * self.b])
