"""Launcher-agnostic rank discovery and process-group bootstrap.

Capability parity with utils/distributed.py:26-177 of the reference (get_rank_info, init_distributed,
cleanup_distributed, is_main_rank, print_rank0) and the 7 inline copies in its scripts, collapsed into one
module.  Differences, by design for a single 8-GPU xGMI node:
  * no mpi4py (not installed, not needed): the MPI launchers are detected from their environment
    variables (OpenMPI, MPICH/PMI, Cray PALS, SLURM) and the rendezvous is always TCPStore (env://);
  * MASTER_ADDR defaults to 127.0.0.1 and MASTER_PORT to 29500 for single-node runs;
  * the backend defaults to "nccl" (= RCCL on ROCm) with a GPU, "gloo" without one -- the device
    binding follows the backend, so the gloo path is genuinely CPU-only (reference defect X5);
  * ``init_process_group`` gets a timeout and eager ``device_id`` (communicators created up front, so
    a broken rank fails at init rather than at the first collective);
  * RCCL failure detection is on by default: ``TORCH_NCCL_ASYNC_ERROR_HANDLING=1`` (a rank whose
    collective times out or errors tears the process down instead of hanging the gang) and the c10d watchdog
    heartbeat ``TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC`` (600 s); user-set values win.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class RankInfo:
    local_rank: int
    world_size: int
    rank: int
    launcher: str

    def __iter__(self):  # allow `local_rank, world_size, rank, launcher = get_rank_info()`
        return iter((self.local_rank, self.world_size, self.rank, self.launcher))


def _int_env(*names: str):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            try:
                return int(v)
            except ValueError:
                pass
    return None


def gpus_per_node() -> int:
    n = _int_env("DPH_GPUS_PER_NODE")
    if n:
        return n
    try:
        c = torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:
        c = 0
    return c if c > 0 else 8


def get_rank_info() -> RankInfo:
    """Priority: torchrun/our launcher -> OpenMPI -> MPICH/PMI (+PALS) -> SLURM -> single process."""
    env = os.environ
    if "RANK" in env and "WORLD_SIZE" in env:
        rank = int(env["RANK"])
        world = int(env["WORLD_SIZE"])
        local = _int_env("LOCAL_RANK")
        if local is None:
            local = rank % gpus_per_node()
        launcher = env.get("DPH_LAUNCHER", "torchrun")
        return RankInfo(local, world, rank, launcher)
    if "OMPI_COMM_WORLD_RANK" in env:
        rank = int(env["OMPI_COMM_WORLD_RANK"])
        world = int(env["OMPI_COMM_WORLD_SIZE"])
        local = _int_env("OMPI_COMM_WORLD_LOCAL_RANK")
        return RankInfo(rank % gpus_per_node() if local is None else local, world, rank, "openmpi")
    if "PMI_RANK" in env and "PMI_SIZE" in env:
        rank = int(env["PMI_RANK"])
        world = int(env["PMI_SIZE"])
        local = _int_env("PMI_LOCAL_RANK", "PALS_LOCAL_RANKID", "MPI_LOCALRANKID")
        return RankInfo(rank % gpus_per_node() if local is None else local, world, rank, "mpich")
    if "SLURM_PROCID" in env and "SLURM_NTASKS" in env:
        rank = int(env["SLURM_PROCID"])
        world = int(env["SLURM_NTASKS"])
        local = _int_env("SLURM_LOCALID")
        return RankInfo(rank % gpus_per_node() if local is None else local, world, rank, "slurm")
    return RankInfo(0, 1, 0, "single")


def default_backend() -> str:
    return "nccl" if torch.cuda.is_available() else "gloo"


def device_for(local_rank: int, backend: str | None = None) -> torch.device:
    backend = backend or default_backend()
    if backend == "nccl" and torch.cuda.is_available():
        n = torch.cuda.device_count()
        if not 0 <= local_rank < n:
            # RCCL cannot put two ranks on one device: a wrong --nproc-per-node / HIP_VISIBLE_DEVICES must fail here,
            # not later inside a collective (gloo ranks may share a GPU: bench.py --backend gloo)
            raise RuntimeError(f"local rank {local_rank} has no GPU of its own ({n} visible); launch at most {n} "
                               f"ranks per node with the nccl (RCCL) backend")
        return torch.device("cuda", local_rank)
    return torch.device("cpu")


# c10d (ProcessGroupNCCL = RCCL on ROCm) failure detection: async error handling + watchdog heartbeat
RCCL_FAILURE_ENV = {"TORCH_NCCL_ASYNC_ERROR_HANDLING": "1", "TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC": "600",
                    "TORCH_NCCL_ENABLE_MONITORING": "1"}


def init_distributed(backend: str | None = None, verbose: bool = True, timeout_s: float = 1800.0,
                     eager: bool = True):
    """Bind the device and create the default process group.

    Returns ``(rank, world_size, local_rank)`` (the reference's utils.distributed.init_distributed order).
    A world of 1 still creates a process group (so collective code paths are exercised).
    """
    info = get_rank_info()
    backend = backend or default_backend()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ["RANK"] = str(info.rank)
    os.environ["WORLD_SIZE"] = str(info.world_size)
    os.environ["LOCAL_RANK"] = str(info.local_rank)
    dev = device_for(info.local_rank, backend)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if backend == "nccl":
        for k, v in RCCL_FAILURE_ENV.items():
            os.environ.setdefault(k, v)
    if not dist.is_initialized():
        kwargs = dict(backend=backend, init_method="env://", rank=info.rank, world_size=info.world_size,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if eager and dev.type == "cuda":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
    if verbose and info.rank == 0:
        print(f"[dph] {info.world_size} rank(s) via {info.launcher}, backend={backend}, "
              f"master={os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}, device={dev.type}", flush=True)
    return info.rank, info.world_size, info.local_rank


def cleanup_distributed():
    if dist.is_initialized():
        dist.destroy_process_group()


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else get_rank_info().rank


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else get_rank_info().world_size


def is_main_rank() -> bool:
    return rank() == 0


def print_rank0(*args, **kwargs):
    if is_main_rank():
        print(*args, **kwargs, flush=True)


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl" and torch.cuda.is_available():
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def verify_min_gpu_count(min_gpus: int = 2) -> bool:
    """utils/logging.py:55-65 of the reference."""
    return torch.cuda.is_available() and torch.cuda.device_count() >= min_gpus


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def hostname() -> str:
    return socket.gethostname()
