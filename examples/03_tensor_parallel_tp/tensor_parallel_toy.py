#!/usr/bin/env python3
"""1-D tensor parallelism of a 64-wide toy model, 10 AdamW iterations (``Iteration i complete``).

Reference: fsdp_tp/tensor_parallel_example.py:76-146 (ToyModel 64 -> 64 -> 64 with ReLU, ``in_proj``
ColwiseParallel + ``out_proj`` RowwiseParallel on a 1-D mesh of all ranks, ``randn(64, 64)`` input seeded per
iteration, AdamW lr 0.25 foreach, output.sum() loss; its 2-D branch is dead code behind ``mesh_1d=True``).
``--dp`` > 1 runs the live version of that 2-D branch: TP inside each dp slice, gradients all-reduced over dp.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/03_tensor_parallel_tp/tensor_parallel_toy.py --dp 2
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D  # noqa: E402
from distributed_pytorch_hpc_amd.models import ToyModel  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.tensor_parallel import (ColwiseParallel, RowwiseParallel,  # noqa: E402
                                                                  parallelize_module)
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.25)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    assert world % args.dp == 0
    mesh = DeviceMesh2D(args.dp, world // args.dp)

    torch.manual_seed(args.seed)
    model = ToyModel(args.dim).to(dev)
    parallelize_module(model, mesh.tp_group, {"in_proj": ColwiseParallel(), "out_proj": RowwiseParallel()})
    engine = DataParallelEngine(model, mesh.dp_group, convert_linears=False)
    engine.configure_optimizer(OptimConfig("adamw", lr=args.lr, weight_decay=0.01))
    losses = []
    for i in range(args.iters):
        torch.manual_seed(i + mesh.dp_rank)   # TP peers share inputs, dp replicas differ
        x = torch.randn(args.dim, args.dim, device=dev)
        loss = model(x).sum()
        loss.backward()
        engine.step()
        engine.zero_grad()
        losses.append(loss.item())
        if rank == 0:
            print(f"Iteration {i} complete (loss {loss.item():.4f})", flush=True)
    engine.synchronize()
    finish(args, {"example": "tensor_parallel_toy", "dp": mesh.dp, "tp": mesh.tp, "losses": losses}, rank)


if __name__ == "__main__":
    main()
