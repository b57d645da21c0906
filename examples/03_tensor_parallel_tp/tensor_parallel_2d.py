#!/usr/bin/env python3
"""2-D tensor parallelism: a stack of pre-LN MLP blocks trained on a (rows x cols) process grid.

The reference only describes 2-D TP (docs/guide/06_tensor_parallel.md:105-128: "2D TP splits along both
dimensions using a 2D GPU grid ... See the scripts for a working example" -- there is none).  Here every weight
is split over both grid dimensions (parallel/tensor_parallel_2d.py): activations are [T/rows, D/cols] blocks,
each Linear all-gathers its input along features over the grid row and its weight over the grid column, and the
backward reduce-scatters both.  Prints per-iteration loss, tokens/s and the per-rank bytes each collective
moves next to what 1-D TP over the same ranks would move (all-reduce of [T, D] twice per block).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/03_tensor_parallel_tp/tensor_parallel_2d.py \
        --rows 2 --cols 4
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
from torch import nn  # noqa: E402

from distributed_pytorch_hpc_amd.parallel.tensor_parallel_2d import (Grid2D, mse_loss_2d,  # noqa: E402
                                                                     parallelize_2d, shard_activation_2d)
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.train.optim import FusedAdamW  # noqa: E402


class Block(nn.Module):
    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.fc1 = nn.Linear(dim, mult * dim)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(mult * dim, dim)

    def forward(self, x):
        return x + self.fc2(self.act(self.fc1(self.norm(x))))


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--rows", type=int, default=None, help="grid rows (default: largest divisor <= sqrt(world))")
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--tokens", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lr", type=float, default=1e-3)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    rows = args.rows or max(r for r in range(1, int(world ** 0.5) + 1) if world % r == 0)
    cols = args.cols or world // rows
    assert rows * cols == world, f"grid {rows}x{cols} != world {world}"
    grid = Grid2D(rows, cols)

    torch.manual_seed(args.seed)
    model = nn.Sequential(*[Block(args.dim) for _ in range(args.depth)]).to(dev)
    parallelize_2d(model, grid)
    opt = FusedAdamW(model.parameters(), lr=args.lr, weight_decay=0.01)

    T, D = args.tokens, args.dim
    g = torch.Generator(device="cpu").manual_seed(args.seed)
    x_full = torch.randn(T, D, generator=g).to(dev)
    y_full = torch.sin(x_full)                      # a smooth target the MLP can fit
    x, y = shard_activation_2d(x_full, grid), shard_activation_2d(y_full, grid)

    losses, times = [], []
    for i in range(args.iters):
        if dev == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        local_loss, loss = mse_loss_2d(model(x), y, grid)
        local_loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        if dev == "cuda":
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        losses.append(float(loss))
        if rank == 0:
            print(f"iter {i}: loss {float(loss):.5f}  {1e3 * times[-1]:.2f} ms", flush=True)

    el = 2 if dev == "cuda" else 4
    # forward all-gather bytes received per rank per block: fc1/fc2 inputs (D and 4D features of T/rows tokens)
    # over the grid row, fc1/fc2 weights (4 D^2 / cols each) over the grid column; 1-D TP: one ring all-reduce
    # of the [T, D] fc2 output over all ranks
    per_block_2d = el * ((cols - 1) / cols * (T / rows) * 5 * D + (rows - 1) / rows * 8 * D * D / cols)
    per_block_1d = el * 2 * T * D * (world - 1) / world
    steady = times[1:] or times
    finish(args, {"example": "tensor_parallel_2d", "grid": [rows, cols], "losses": losses,
                  "tokens_per_s": T / (sum(steady) / len(steady)),
                  "fwd_bytes_per_rank_per_block_2d": per_block_2d,
                  "fwd_bytes_per_rank_per_block_1d_tp": per_block_1d}, rank)


if __name__ == "__main__":
    main()
