"""Every example driver (examples/*) runs end-to-end under torchrun on CPU/gloo and prints its JSON summary.

Mirrors how the reference is exercised (tests/run_tests.sh launching the drivers with each backend), on tiny
configurations so the whole set stays within the CPU test budget.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")

CASES = [
    ("01_data_parallel_ddp/ddp_basic.py", 2, ["3", "2", "--snapshot-path", "{tmp}/snap.pt"]),
    ("01_data_parallel_ddp/distributed_dataloader.py", 2, ["--epochs", "2"]),
    ("01_data_parallel_ddp/ddp_unet.py", 2, ["--lat", "33", "--lon", "40", "--channels", "3", "--base-dim", "8",
                                            "--steps-per-epoch", "2"]),
    ("02_fully_sharded_fsdp/fsdp_resnet.py", 2, ["--arch", "resnet18", "--batch-size", "4", "--steps-per-epoch",
                                                 "2", "--test-steps", "1", "--use-amp"]),
    ("02_fully_sharded_fsdp/fsdp_unet.py", 2, ["--lat", "33", "--lon", "40", "--channels", "3", "--base-dim", "8",
                                               "--steps-per-epoch", "2", "--checkpoint", "{tmp}/full.pt"]),
    ("03_tensor_parallel_tp/device_mesh_basics.py", 4, []),
    ("03_tensor_parallel_tp/basic_tensor_parallel.py", 2, ["--iters", "3"]),
    ("03_tensor_parallel_tp/tensor_parallel_toy.py", 4, ["--dp", "2", "--iters", "3"]),
    ("03_tensor_parallel_tp/tensor_parallel_2d.py", 4, ["--iters", "3", "--dim", "64", "--tokens", "64"]),
    ("03_tensor_parallel_tp/tensor_parallel_vit.py", 2, ["--tp", "2", "--steps-per-epoch", "2", "--epochs", "1",
                                                         "--channels", "3", "--depth", "2"]),
    ("04_pipeline_parallel_pp/manual_model_split.py", 2, ["--train", "--steps", "2"]),
    ("04_pipeline_parallel_pp/pipeline_schedules.py", 2, ["--steps", "2", "--warmup", "1"]),
    ("04_pipeline_parallel_pp/pipeline_training.py", 2, ["--steps", "2", "--warmup", "1", "--vocab", "1000",
                                                         "--seq-len", "32", "--batch", "8"]),
    ("05_sequence_context_parallel/context_parallel_llama.py", 2, ["--mode", "ulysses", "--seq-len", "64",
                                                                   "--steps", "2", "--model", "tiny"]),
    ("05_sequence_context_parallel/context_parallel_llama.py", 2, ["--mode", "ring", "--seq-len", "64",
                                                                   "--steps", "2", "--model", "tiny"]),
    ("06_hybrid_parallelism/fsdp_tp_hybrid.py", 4, ["--tp", "2", "--iters", "2", "--batch", "2", "--seq-len",
                                                    "32", "--model", "tiny"]),
    ("06_hybrid_parallelism/fsdp_tp_hybrid.py", 4, ["--tp", "2", "--iters", "2", "--batch", "2", "--seq-len",
                                                    "32", "--model", "tiny", "--async-tp", "2"]),
    ("06_hybrid_parallelism/three_d_parallel.py", 4, ["--pp", "2", "--tp", "2", "--iters", "2", "--batch", "4",
                                                      "--seq-len", "32", "--model", "tiny"]),
    ("07_domain_parallel/domain_parallel_unet.py", 2, ["--lat", "32", "--lon", "32", "--channels", "3",
                                                       "--base-dim", "8", "--steps", "2", "--check"]),
    ("08_serving/generate_llama.py", 2, ["--batch", "2", "--prompt-len", "8", "--max-new", "6"]),
    ("08_serving/generate_llama.py", 1, ["--batch", "3", "--prompt-len", "5", "--max-new", "4", "--temperature",
                                         "0.8", "--top-k", "20"]),
    ("resnet_benchmark.py", 2, ["--arch", "resnet18", "--batch-size", "4", "--image-size", "32", "--epochs", "2",
                                "--steps-syn", "1"]),
]


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(script, nproc, args, tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(EX, script), "--device", "cpu"]
    cmd += [a.format(tmp=str(tmp_path)) for a in args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, f"{script} failed:\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:]
    return json.loads(lines[-1])


@pytest.mark.parametrize("script,nproc,args", CASES, ids=[f"{c[0].split('/')[-1][:-3]}-{i}" for i, c in enumerate(CASES)])
def test_example_runs(script, nproc, args, tmp_path):
    out = _run(script, nproc, args, tmp_path)
    assert "example" in out


def test_ddp_basic_resumes_from_snapshot(tmp_path):
    first = _run("01_data_parallel_ddp/ddp_basic.py", 2, ["2", "2", "--snapshot-path", "{tmp}/snap.pt"], tmp_path)
    assert first["epochs"] == 2 and os.path.exists(tmp_path / "snap.pt")
    second = _run("01_data_parallel_ddp/ddp_basic.py", 2, ["4", "2", "--snapshot-path", "{tmp}/snap.pt"], tmp_path)
    assert second["epochs"] == 2   # resumed at epoch 2, ran epochs 2 and 3 only


def test_fsdp_resnet_on_cifar_binary_files(tmp_path):
    """--data-dir: the CIFAR-10 binary distribution (fake records here; no download) through the device loader."""
    import numpy as np

    from distributed_pytorch_hpc_amd.data.cifar import write_cifar_bin

    rng = np.random.default_rng(0)
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        write_cifar_bin(str(d / name), rng.integers(0, 256, (8, 32, 32, 3), dtype=np.uint8),
                        rng.integers(0, 10, 8).astype(np.uint8))
    out = _run("02_fully_sharded_fsdp/fsdp_resnet.py", 2, ["--arch", "resnet18", "--batch-size", "4",
                                                           "--steps-per-epoch", "3", "--test-steps", "2",
                                                           "--data-dir", str(d)], tmp_path)
    assert out["example"] == "fsdp_resnet" and out["test"]["samples"] == 8   # the 8 test images, 4 per rank
    # the ResNet benchmark driver (scripts/main.py parity) on the same files: full epochs of 40 / 2 / 4 = 5 steps
    out = _run("resnet_benchmark.py", 2, ["--arch", "resnet18", "--batch-size", "4", "--epochs", "1", "--eval-steps",
                                          "1", "--data-dir", str(d)], tmp_path)
    assert out["example"] == "resnet_benchmark" and out["eval"]["samples"] == 8
