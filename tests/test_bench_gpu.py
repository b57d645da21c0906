"""bench.py's N > 1 path on GPU tensors: two ranks share one MI355X over gloo (RCCL needs a GPU per rank), tiny
Llama, HIP kernels.  Same contract checks as tests/test_bench.py; the round-end driver runs this code path with RCCL
on 2, 4 and 8 GPUs."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("fp8", [False, True])
def test_bench_two_ranks_share_one_gpu(tmp_path, fp8):
    """fp8: the opt-in FP8-GEMM mode under the sharded engine (weight gradients written into ZeRO-2 buckets)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--model", "tiny", "--seq-len", "128", "--micro-batch", "2",
           "--steps", "2", "--warmup", "1", "--quiet"] + (["--fp8"] if fp8 else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=str(tmp_path),
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1, p.stdout
    r = recs[0]
    assert r["n_gpus"] == 2 and r["dtype"] == ("bf16+fp8-gemm" if fp8 else "bf16") and r["value"] > 0
    assert abs(r["loss_last"] - r["loss_first_warmup"]) < 2.0
    assert r["config"]["parallelism"] == "fsdp2" and r["config"]["global_batch"] == 4
    assert r["config"]["kernels"] == "dph"
    assert r["preflight_ok"] is True and r["param_checksum_ok"] is True


def test_bench_tp_layout_two_ranks_share_one_gpu(tmp_path):
    """--layout tp (BASELINE config 3's TP + SP + loss-parallel plan) on GPU tensors: two gloo ranks, one MI355X."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--layout", "tp", "--model", "tiny8", "--seq-len", "128",
           "--micro-batch", "2", "--steps", "2", "--warmup", "1", "--quiet"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=str(tmp_path),
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0, p.stderr[-3000:]
    r = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")][0]
    assert r["config"]["parallelism"] == "tp2" and r["dtype"] == "bf16" and r["value"] > 0
    assert abs(r["loss_last"] - r["loss_first_warmup"]) < 2.0


def test_bench_more_gpus_than_visible_fails(tmp_path):
    """On a box with fewer GPUs than --gpus, bench.py must exit non-zero instead of timing fewer ranks."""
    import torch

    n = torch.cuda.device_count()
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--model", "tiny", "--quiet"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=str(tmp_path), env=env)
    assert p.returncode == 2, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("layout", ["resnet-fsdp", "unet-ddp"])
def test_bench_one_rank_conv_layouts_replay_graph(tmp_path, layout):
    """The one-rank resnet-fsdp / unet-ddp layouts replay each timed step as one HIP graph by default (captured in the
    warm-up); the loss stays finite and the line says so."""
    extra = (["--arch", "resnet18", "--image-size", "64", "--micro-batch", "8"] if layout == "resnet-fsdp"
             else ["--micro-batch", "1"])
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--layout", layout, "--steps", "3", "--warmup", "2",
           "--quiet", "--no-telemetry"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    r = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")][0]
    assert r["n_gpus"] == 1 and r["value"] > 0 and "graph" in r, r
    assert r["loss_last"] == r["loss_last"]   # not NaN


def test_bench_resnet50_fsdp_two_ranks_share_one_gpu(tmp_path):
    """ResNet-50 under the FSDP engine at world 2 (two gloo ranks on one MI355X) with every round-6 BatchNorm path on
    (reductions in the consumers' epilogues, masked residual hand-off, projection-shortcut dual BatchNorm): the step
    runs on both ranks and the loss stays finite (the parameters are sharded, so there is no replica checksum)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--layout", "resnet-fsdp", "--arch", "resnet50", "--image-size", "64",
           "--micro-batch", "4", "--steps", "2", "--warmup", "1", "--quiet", "--no-telemetry"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=str(tmp_path),
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0, p.stderr[-3000:]
    r = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")][0]
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["loss_last"] == r["loss_last"]
    assert r["config"]["parallelism"] == "fsdp2"
