#!/usr/bin/env python3
"""Environment checker for an MI355X node (capability parity with tests/check_environment.py, tests/test_env.py and
tests/print_hostinfo.py of the reference, re-targeted from CUDA/NCCL/Slingshot to ROCm/RCCL/xGMI).

Single process: versions (torch, HIP runtime, RCCL), GPUs (name, arch, CUs, HBM), the in-tree HIP extension
(is it built for gfx950 and loadable, does a kernel run), xGMI topology from ``amd-smi``/``rocm-smi`` when
available, relevant env vars (NCCL_/RCCL_/HSA_/HIP_), and a world-size-1 collective smoke test.
Distributed (under torchrun / our launcher): all_gather_object of every rank's host + device, rank -> GPU map,
and an all-reduce check of sum(range(world)).  Prints a ✓/✗ summary; exit code 1 on any failure.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402


def _run(cmd):
    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=30).stdout.strip()
    except Exception as e:  # pragma: no cover
        return f"<{e}>"


def local_report() -> dict:
    r = {"host": rt.hostname(), "torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
         "gloo": dist.is_gloo_available(), "nccl(rccl)": dist.is_nccl_available(), "mpi": dist.is_mpi_available(),
         "gpus": []}
    try:
        r["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
    except Exception:
        r["rccl_version"] = None
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            r["gpus"].append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", "?"),
                              "cus": p.multi_processor_count, "hbm_gb": round(p.total_memory / 1e9, 1)})
    from distributed_pytorch_hpc_amd.ops import _lib

    r["native_extension"] = {"path": _lib.SO_PATH, "exists": os.path.exists(_lib.SO_PATH), "loaded": _lib.load()}
    if torch.cuda.is_available() and r["native_extension"]["loaded"]:
        from distributed_pytorch_hpc_amd import ops

        x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
        w = torch.ones(256, device="cuda", dtype=torch.bfloat16)
        err = (ops.rms_norm(x, w) - ops.rmsnorm_reference(x, w, 1e-5)).abs().max().item()
        r["native_extension"]["rmsnorm_max_err"] = err
    if shutil.which("amd-smi"):
        r["xgmi_topology"] = _run(["amd-smi", "topology"])[:4000]
    elif shutil.which("rocm-smi"):
        r["xgmi_topology"] = _run(["rocm-smi", "--showtopotype"])[:4000]
    r["env"] = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_", "ROCR_"))}
    # rank -> GPU -> NUMA -> CPU map the launcher applies (runtime/device.py), plus this process's actual affinity
    from distributed_pytorch_hpc_amd.runtime import device

    nproc = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "0")) or 0) or \
        max(1, len(device.gpus()))
    r["gpu_numa"] = [{"gpu": g.index, "pci": g.bdf, "numa": g.numa_node, "local_cpus": len(g.local_cpus)}
                     for g in device.gpus()]
    r["cpu_binding_plan"] = device.describe(device.plan(nproc)).splitlines()
    try:
        r["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        r["affinity"] = None
    r["cpu_bind_env"] = os.environ.get("DPH_CPU_BIND")
    return r


def main():
    checks = []
    rep = local_report()
    checks.append(("torch imports", True))
    checks.append(("HIP runtime present", rep["hip"] is not None))
    if torch.cuda.is_available():
        checks.append(("GPU visible", len(rep["gpus"]) > 0))
        checks.append(("gfx950 (MI355X)", any("gfx950" in g["arch"] for g in rep["gpus"])))
        checks.append(("native HIP extension loads", bool(rep["native_extension"]["loaded"])))
        checks.append(("native kernel numerics", rep["native_extension"].get("rmsnorm_max_err", 1.0) < 0.05))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:
        rank, world, local = rt.init_distributed(verbose=False)
        infos = [None] * world
        dist.all_gather_object(infos, {"rank": rank, "host": rep["host"], "local_rank": local,
                                       "numa": os.environ.get("DPH_NUMA_NODE"), "cpus": rep["affinity"],
                                       "device": torch.cuda.current_device() if torch.cuda.is_available() else "cpu"})
        dev = rt.device_for(local)
        t = torch.tensor([float(rank)], device=dev)
        dist.all_reduce(t)
        ok = t.item() == world * (world - 1) / 2
        checks.append((f"all_reduce over {world} ranks", ok))
        rep["ranks"] = infos
    else:
        rank = 0
        # world-size-1 process group smoke test (tests/test_env.py of the reference)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(rt.free_port()))
        os.environ.update(RANK="0", WORLD_SIZE="1")
        rt.init_distributed(verbose=False)
        dev = rt.device_for(0)
        t = torch.tensor([1.0, 2.0], device=dev)
        dist.all_reduce(t)
        checks.append(("world-1 all_reduce", t.tolist() == [1.0, 2.0]))
    if rank == 0:
        print(json.dumps(rep, indent=1, default=str))
        for name, ok in checks:
            print(("✓ " if ok else "✗ ") + name)
    rt.cleanup_distributed()
    sys.exit(0 if all(ok for _, ok in checks) else 1)


if __name__ == "__main__":
    main()
