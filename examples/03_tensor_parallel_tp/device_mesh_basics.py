#!/usr/bin/env python3
"""Process meshes: 1-D mesh of all ranks, 2-D (dp, tp) mesh, sub-group slicing, all-reduce sanity check.

Reference: scripts/03_tensor_parallel_tp/01_device_mesh_basics.py (``init_device_mesh("cuda", (world,))``, 2-D
``(dp, tp)`` with names ("dp", "tp"), last dim fastest-varying, ``mesh["tp"]`` / ``mesh["dp"]`` slicing, all-reduce
of ``rank`` checked against ``sum(range(W))``, L29-89).

On one MI355X node all 8 GPUs are pairwise one xGMI hop apart, so any (dp, tp) factorisation is topologically
equivalent; tp stays fastest-varying so that multi-node meshes keep TP inside a node.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/03_tensor_parallel_tp/device_mesh_basics.py --tp 4
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D, Mesh, mesh_sanity_check  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--tp", type=int, default=None, help="tp size of the 2-D mesh (default: 2 if world is even)")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    mesh1 = Mesh((world,), ("world",))
    tot = torch.tensor([float(rank)], device=dev)
    if world > 1:
        dist.all_reduce(tot)
    ok1 = tot.item() == sum(range(world))
    tp = args.tp or (2 if world % 2 == 0 else 1)
    assert world % tp == 0, f"world {world} not divisible by tp {tp}"
    mesh2 = DeviceMesh2D(world // tp, tp)
    checks = mesh_sanity_check(mesh2, dev)
    ok2 = all(got == exp for got, exp in checks.values())
    line = (f"rank {rank}: 1-D {mesh1.shape} | 2-D (dp={mesh2.dp}, tp={mesh2.tp}) coords dp={mesh2.dp_rank} "
            f"tp={mesh2.tp_rank} | tp group {mesh2.group_ranks['tp']} | dp group {mesh2.group_ranks['dp']}")
    gathered = [None] * world
    if world > 1:
        dist.all_gather_object(gathered, line)
    else:
        gathered = [line]
    if rank == 0:
        for g in gathered:
            print(g, flush=True)
        print(f"all_reduce(rank) = {tot.item():.0f} (expected {sum(range(world))}): {'OK' if ok1 else 'FAIL'}")
    summary = {"example": "device_mesh_basics", "world": world, "dp": mesh2.dp, "tp": mesh2.tp,
               "world_allreduce_ok": ok1, "submesh_allreduce_ok": ok2}
    finish(args, summary, rank)
    if not (ok1 and ok2):
        sys.exit(1)


if __name__ == "__main__":
    main()
