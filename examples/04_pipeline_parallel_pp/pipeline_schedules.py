#!/usr/bin/env python3
"""GPipe vs 1F1B on a 4-block MLP: step time, bubble fraction and in-flight activation count.

Reference: scripts/04_pipeline_parallel_pp/02_pipeline_schedules.py:45-212 (FourBlockMLP dim 512 split into
one block per rank with ``pipeline(..., split_spec)``, ScheduleGPipe vs Schedule1F1B timed, "theoretical bubble"
printed as (S-1)/M -- reference defect X4).

Here both schedules run full training steps (forward + backward, sum loss) through parallel/pipeline.py; the
bubble is the idle FRACTION (S-1)/(M+S-1), identical for both schedules; 1F1B's advantage is its peak
number of live micro-batch activations on stage s: min(S-s, M) instead of M.

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/04_pipeline_parallel_pp/pipeline_schedules.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.models import FourBlockMLP  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, bubble_fraction, split_sequential  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.utils.metrics import sync  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--microbatches", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    torch.manual_seed(args.seed)
    full = FourBlockMLP(args.dim).as_sequential()
    stage_mod = split_sequential(full, world, rank).to(dev)
    results = {}
    for sched_name in ("gpipe", "1f1b"):
        sched = PipelineSchedule(stage_mod, rank, world, args.microbatches, loss_fn=None, schedule=sched_name,
                                 device=dev)
        x = torch.randn(args.batch, args.dim, device=dev) if rank == 0 else None
        for i in range(args.warmup + args.steps):
            if i == args.warmup:
                sync()
                if world > 1:
                    dist.barrier()
                t0 = time.perf_counter()
            sched.step(inputs=x)
            for p in stage_mod.parameters():
                p.grad = None
        sync()
        if world > 1:
            dist.barrier()
        dt = (time.perf_counter() - t0) / args.steps
        results[sched_name] = dt
        if rank == 0:
            print(f"{sched_name:6s}: {1000 * dt:.3f} ms/step", flush=True)
    bub = bubble_fraction(world, args.microbatches)
    if rank == 0:
        print(f"bubble (idle fraction) = (S-1)/(M+S-1) = {bub:.3f} for both schedules; peak live micro-batches "
              f"on stage 0: GPipe {args.microbatches}, 1F1B {min(world, args.microbatches)}", flush=True)
    summary = {"example": "pipeline_schedules", "stages": world, "microbatches": args.microbatches,
               "ms_per_step": {k: 1000 * v for k, v in results.items()}, "bubble_fraction": bub}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
