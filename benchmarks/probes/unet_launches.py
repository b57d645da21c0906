#!/usr/bin/env python3
"""Which ATen (non-framework) device kernels the SimpleUNet DDP step launches, and from where: torch.profiler over
a few steps of the bench workload (train/bench_layouts.py build_unet_ddp), grouped by the 6 innermost Python frames.

    python benchmarks/probes/unet_launches.py [--steps 3]
"""
import argparse
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from distributed_pytorch_hpc_amd.train.bench_layouts import build_unet_ddp

    args = types.SimpleNamespace(unet_precision="bf16", micro_batch=4, bucket_mb="calibrate")
    dev = torch.device("cuda")
    import torch.distributed as dist

    from distributed_pytorch_hpc_amd.runtime.env import free_port

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    try:
        wl = build_unet_ddp(args, 0, 1, dev, print)
    except AttributeError as e:   # bench args the builder reads that this probe did not set
        raise SystemExit(f"build_unet_ddp needs another bench argument: {e}")
    for i in range(3):
        wl.step(i)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(a.steps):
            wl.step(i)
        torch.cuda.synchronize()
    table = prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=60, max_name_column_width=60)
    print(table)


if __name__ == "__main__":
    main()
