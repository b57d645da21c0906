#!/usr/bin/env python3
"""Megatron 1-D tensor parallelism on a toy MLP (Colwise -> ReLU -> Rowwise), checked against one device.

Reference: scripts/03_tensor_parallel_tp/02_basic_tensor_parallel.py:46-92 (ToyMLP 16 -> 64 -> 16, ``in_proj``
ColwiseParallel, ``out_proj`` RowwiseParallel on a 1-D mesh of all ranks, ``randn(8, 16)`` seeded per
iteration so every TP rank sees the same input, AdamW lr 1e-3, loss = output.sum(), loss printed per iter).

MI355X version: parallel/tensor_parallel.py shards the weights explicitly (no DTensor dispatch): the column
shard's GEMM needs no communication, the row shard's partial sums are all-reduced over the TP group (RCCL).
``--check`` replays the same iterations on an unsharded copy and asserts the losses match.

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/03_tensor_parallel_tp/basic_tensor_parallel.py
"""
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.models import ToyMLP  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.tensor_parallel import (ColwiseParallel, RowwiseParallel,  # noqa: E402
                                                                  parallelize_module)
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--in-dim", type=int, default=16)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--check", action=__import__("argparse").BooleanOptionalAction, default=True)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    tp_group = dist.group.WORLD if world > 1 else None

    torch.manual_seed(args.seed)
    model = ToyMLP(args.in_dim, args.hidden, args.in_dim).to(dev)
    ref = copy.deepcopy(model) if args.check else None
    parallelize_module(model, tp_group, {"in_proj": ColwiseParallel(), "out_proj": RowwiseParallel()})
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=args.lr) if ref is not None else None
    losses, max_err = [], 0.0
    for i in range(args.iters):
        torch.manual_seed(i)                      # same input on every TP rank
        x = torch.randn(args.batch, args.in_dim, device=dev)
        loss = model(x).sum()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
        if ref is not None:
            rl = ref(x).sum()
            ref_opt.zero_grad()
            rl.backward()
            ref_opt.step()
            max_err = max(max_err, abs(rl.item() - loss.item()) / max(abs(rl.item()), 1.0))
        if rank == 0:
            print(f"iter {i}: loss {loss.item():.6f}", flush=True)
    summary = {"example": "basic_tensor_parallel", "tp": world, "losses": losses}
    if ref is not None:
        summary["max_rel_err_vs_unsharded"] = max_err
        assert max_err < 1e-4, f"TP diverged from the unsharded model: {max_err}"
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
