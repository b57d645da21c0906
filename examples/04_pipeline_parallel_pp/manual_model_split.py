#!/usr/bin/env python3
"""Manual pipeline split: one Linear stage per rank, micro-batches passed with blocking send/recv.

Reference: scripts/04_pipeline_parallel_pp/01_manual_model_split.py:53-157 (stages 128->256->256->256->64 on
exactly 4 ranks, batch 32 split into 4 micro-batches of 8, forward-only ``dist.send`` / ``dist.recv`` chain,
shapes printed).

MI355X version: any number of ranks >= 2 (the dims list is stretched/cut to the world size), the shapes travel
with each micro-batch, and ``--train`` also runs the backward chain (gradients sent back stage to stage) with a
per-stage SGD step -- the reference stops at the forward.  Every neighbouring pair is one xGMI hop.

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/04_pipeline_parallel_pp/manual_model_split.py --train
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.models import StageModule  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.pipeline import P2P  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def stage_dims(world):
    base = [128, 256, 256, 256, 64]
    if world + 1 <= len(base):
        return base[:world] + [64]
    return [128] + [256] * (world - 1) + [64]


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--microbatches", type=int, default=4)
    ap.add_argument("--train", action="store_true", help="also pipeline the backward pass + SGD step")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    assert world >= 2, "the manual pipeline needs at least 2 ranks"
    dims = stage_dims(world)
    torch.manual_seed(args.seed + rank)
    stage = StageModule(dims[rank], dims[rank + 1], is_last=(rank == world - 1)).to(dev)
    opt = torch.optim.SGD(stage.parameters(), lr=1e-2)
    p2p = P2P(None, rank, world, dev)
    log = []
    for step in range(args.steps):
        inputs = []
        outputs = []
        if rank == 0:
            torch.manual_seed(1000 + step)
            x_full = torch.randn(args.batch, dims[0], device=dev)
            micro = list(x_full.chunk(args.microbatches))
        for i in range(args.microbatches):
            x = micro[i] if rank == 0 else p2p.recv_forward(with_header=(i == 0))
            if args.train and rank > 0:
                x.requires_grad_(True)
            y = stage(x)
            inputs.append(x)
            outputs.append(y)
            if rank < world - 1:
                p2p.send_forward(y, with_header=(i == 0))
            if step == 0:
                log.append(f"stage {rank} mb {i}: in {tuple(x.shape)} -> out {tuple(y.shape)}")
        loss = None
        if args.train:
            opt.zero_grad()
            for i in reversed(range(args.microbatches)):
                if rank == world - 1:
                    mb_loss = outputs[i].pow(2).mean() / args.microbatches
                    loss = mb_loss.detach() if loss is None else loss + mb_loss.detach()
                    mb_loss.backward()
                else:
                    outputs[i].backward(p2p.recv_backward(outputs[i]))
                if rank > 0:
                    p2p.send_backward(inputs[i].grad)
            opt.step()
        if rank == world - 1 and loss is not None:
            print(f"step {step}: loss {loss.item():.6f}", flush=True)
    lines = [None] * world
    dist.all_gather_object(lines, log)
    if rank == 0:
        for ls in lines:
            for line in ls:
                print(line, flush=True)
    summary = {"example": "manual_model_split", "stages": world, "dims": dims, "microbatches": args.microbatches,
               "trained": args.train}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
