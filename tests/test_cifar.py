"""CIFAR-10 binary reader + on-device batch assembly (data/cifar.py, csrc/imageaug.hip)."""
import numpy as np
import pytest
import torch

from distributed_pytorch_hpc_amd.data.cifar import (CIFAR10, MEAN, STD, CIFARDeviceLoader, augment_reference,
                                                    write_cifar_bin)


def _fake_split(root, n_per_batch=40, seed=0):
    rng = np.random.default_rng(seed)
    allimg, alllab = [], []
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        img = rng.integers(0, 256, (n_per_batch, 32, 32, 3), dtype=np.uint8)
        lab = rng.integers(0, 10, n_per_batch).astype(np.uint8)
        write_cifar_bin(str(root / name), img, lab)
        if name != "test_batch.bin":
            allimg.append(img)
            alllab.append(lab)
    return np.concatenate(allimg), np.concatenate(alllab)


def test_reader_roundtrip(tmp_path):
    img, lab = _fake_split(tmp_path)
    ds = CIFAR10(str(tmp_path), train=True)
    assert len(ds) == 200 and np.array_equal(ds.images, img) and np.array_equal(ds.labels, lab.astype(np.int64))
    x, y = ds[7]
    assert x.shape == (32, 32, 3) and x.dtype == torch.uint8 and y == int(lab[7])
    assert len(CIFAR10(str(tmp_path), train=False)) == 40
    with pytest.raises(FileNotFoundError):
        CIFAR10(str(tmp_path / "nope"))


def test_reference_transform_semantics():
    """RandomCrop(32, padding=4) + flip + ToTensor + Normalize, element by element."""
    torch.manual_seed(0)
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    prm = torch.tensor([[0, 8, 1], [4, 4, 0]], dtype=torch.int32)
    out = augment_reference(img, prm, MEAN, STD)
    m, s = torch.tensor(MEAN), torch.tensor(STD)
    # sample 1: centred crop, no flip -> plain normalisation
    assert torch.allclose(out[1], (img[1].permute(2, 0, 1).float() / 255 - m.view(3, 1, 1)) / s.view(3, 1, 1),
                          atol=1e-6)
    # sample 0: dy=0 (4 rows of padding on top), dx=8 (shifted left by 4), then flipped
    y, x = 10, 5
    sx = (31 - x) + 8 - 4
    want = (img[0, y - 4, sx].float() / 255 - m) / s if 0 <= sx < 32 else (-m / s)
    assert torch.allclose(out[0, :, y, x], want, atol=1e-6)
    assert torch.allclose(out[0, :, 2, 3], -m / s, atol=1e-6)   # row 2 comes from the zero padding


def test_device_loader_sharding_cpu(tmp_path):
    _fake_split(tmp_path, n_per_batch=25)   # 125 training images, not divisible by 2
    ds = CIFAR10(str(tmp_path))
    seen = []
    for r in range(2):
        ld = CIFARDeviceLoader(ds, batch_size=16, device="cpu", dp_rank=r, dp_size=2, augment=False, seed=3,
                               drop_last=False)
        ld.set_epoch(1)
        batches = list(ld)
        assert len(batches) == len(ld) == 4 and batches[-1][0].shape[0] == 63 - 48
        for x, y in batches:
            assert x.shape[1:] == (3, 32, 32) and x.dtype == torch.float32
            seen.append(y)
    # DistributedSampler padding: 126 slots over 2 ranks cover every sample at least once
    assert torch.cat(seen).numel() == 126
    ld = CIFARDeviceLoader(ds, batch_size=8, device="cpu", augment=False, shuffle=False)
    x, y = next(iter(ld))
    ref = augment_reference(torch.from_numpy(ds.images[:8]), None, MEAN, STD)
    assert torch.allclose(x, ref) and torch.equal(y, torch.from_numpy(ds.labels[:8]))


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_augment_kernel_matches_reference(dph_native, channels_last, dtype):
    torch.manual_seed(1)
    images = torch.randint(0, 256, (300, 32, 32, 3), dtype=torch.uint8, device="cuda")
    idx = torch.randint(0, 300, (77,), device="cuda")
    prm = torch.cat([torch.randint(0, 9, (77, 2), device="cuda", dtype=torch.int32),
                     torch.randint(0, 2, (77, 1), device="cuda", dtype=torch.int32)], 1).contiguous()
    mean = torch.tensor(MEAN, device="cuda")
    inv = 1.0 / torch.tensor(STD, device="cuda")
    out = dph_native.image_augment(images, idx, prm, mean, inv, 4, channels_last, dtype == torch.bfloat16)
    ref = augment_reference(images[idx], prm, MEAN, STD, 4, channels_last, torch.float32)
    assert out.shape == (77, 3, 32, 32) and out.dtype == dtype
    assert out.is_contiguous(memory_format=torch.channels_last) == channels_last
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert (out.float() - ref).abs().max().item() < tol
    plain = dph_native.image_augment(images, idx, None, mean, inv, 4, channels_last, False)
    assert torch.allclose(plain, augment_reference(images[idx], None, MEAN, STD), atol=1e-5)


@pytest.mark.gpu
def test_device_loader_gpu_reproducible(dph_native, tmp_path):
    _fake_split(tmp_path)
    ds = CIFAR10(str(tmp_path))
    a = CIFARDeviceLoader(ds, 32, "cuda", seed=5, dtype=torch.bfloat16, channels_last=True)
    b = CIFARDeviceLoader(ds, 32, "cuda", seed=5, dtype=torch.bfloat16, channels_last=True)
    for (xa, ya), (xb, yb) in zip(a, b):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
    assert xa.is_contiguous(memory_format=torch.channels_last)
