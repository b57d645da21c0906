"""Launcher: env contract, gang teardown on a rank failure, restart + resume (SURVEY.md §5.3 fault injection)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kill_a_rank_then_resume(tmp_path):
    cmd = [sys.executable, "-m", "distributed_pytorch_hpc_amd.runtime.launch", "--nproc", "4", "--max-restarts", "1",
           "--timeout", "240", "--grace", "5", "--log-dir", str(tmp_path / "logs"),
           os.path.join(ROOT, "tests", "scripts", "fault_train.py"), str(tmp_path)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "rank 2 exited with 3" in r.stderr and "restarting" in r.stderr
    for k in range(4):
        start, attempt = open(tmp_path / f"DONE.{k}").read().split()
        assert start == "2" and attempt == "1"


def test_failure_without_restart_propagates(tmp_path):
    cmd = [sys.executable, "-m", "distributed_pytorch_hpc_amd.runtime.launch", "--nproc", "4", "--timeout", "240",
           "--grace", "5", os.path.join(ROOT, "tests", "scripts", "fault_train.py"), str(tmp_path)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3
    assert not any(f.startswith("DONE") for f in os.listdir(tmp_path))


def test_rank_detection_precedence(monkeypatch):
    from distributed_pytorch_hpc_amd.runtime.env import get_rank_info

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "PMI_RANK",
              "PMI_SIZE", "SLURM_PROCID", "SLURM_NTASKS", "DPH_LAUNCHER"):
        monkeypatch.delenv(k, raising=False)
    assert tuple(get_rank_info()) == (0, 1, 0, "single")
    monkeypatch.setenv("PMI_RANK", "5")
    monkeypatch.setenv("PMI_SIZE", "8")
    monkeypatch.setenv("PALS_LOCAL_RANKID", "1")
    assert tuple(get_rank_info()) == (1, 8, 5, "mpich")
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "3")
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "4")
    assert get_rank_info().launcher == "openmpi"
    monkeypatch.setenv("RANK", "2")
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_RANK", "2")
    assert tuple(get_rank_info()) == (2, 16, 2, "torchrun")


def test_utils_facade_has_reference_names():
    """utils/__init__.py of the reference re-exports these; scripts written against it import them by name."""
    import distributed_pytorch_hpc_amd.utils as u

    for name in ("get_rank_info", "init_distributed", "cleanup_distributed", "is_main_rank", "print_rank0",
                 "get_logger", "rank_log", "verify_min_gpu_count", "training_profiler", "print_profiler_summary",
                 "save_checkpoint", "load_checkpoint", "TrainingConfig", "redirect"):
        assert callable(getattr(u, name)), name


def test_device_for_refuses_shared_gpu_under_rccl(monkeypatch):
    """nccl (RCCL) ranks need a GPU each: local rank >= visible GPUs fails at startup; gloo ranks stay on the CPU
    device (several may then share one GPU explicitly, bench.py --backend gloo)."""
    import pytest

    from distributed_pytorch_hpc_amd.runtime import env as rt

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    assert rt.device_for(1, "nccl") == torch.device("cuda", 1)
    with pytest.raises(RuntimeError, match="no GPU of its own"):
        rt.device_for(2, "nccl")
    assert rt.device_for(5, "gloo").type == "cpu"
