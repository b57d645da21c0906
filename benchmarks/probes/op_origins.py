#!/usr/bin/env python3
"""Where do a bench layout's small ATen ops come from?  Runs a few steps of a ``bench.py --layout`` workload under
torch.profiler (with_stack) and prints, per ATen op of interest (copy_, fill_, zero_, ...), the count per step and the
innermost framework source lines that issued it.

    python benchmarks/probes/op_origins.py --layout resnet-fsdp [--ops aten::copy_,aten::fill_] [--steps 2]
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench
    from distributed_pytorch_hpc_amd.train.bench_layouts import BUILDERS

    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet-fsdp")
    ap.add_argument("--ops", default="aten::copy_,aten::fill_,aten::zero_,aten::zeros,aten::add_,aten::contiguous")
    ap.add_argument("--steps", type=int, default=2)
    a, rest = ap.parse_known_args()
    args = bench.parse(["--layout", a.layout, "--no-dist"] + rest)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = BUILDERS[a.layout](args, 0, 1, dev, lambda m: None)
    for i in range(3):
        wl.step(i)
    torch.cuda.synchronize()
    want = set(a.ops.split(","))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True,
                                record_shapes=True) as prof:
        for i in range(a.steps):
            wl.step(3 + i)
        torch.cuda.synchronize()
    by = collections.defaultdict(collections.Counter)
    for ev in prof.events():
        if ev.name not in want:
            continue
        # nested ops (copy_ under aten::to / contiguous, or under an autograd node) carry no stack themselves: walk
        # up the parents, keeping their names, to the first one that has framework frames
        chain, e, frames = [], ev, []
        while e is not None and not frames:
            frames = [f for f in (e.stack or []) if "distributed_pytorch_hpc_amd" in f or "bench" in f]
            if not frames:
                chain.append(e.name)
                e = e.cpu_parent
        key = " < ".join(chain[1:4]) + (" | " if chain[1:] else "") + \
            (" <- ".join(f.split(ROOT + "/")[-1] for f in frames[:3]) or "(no framework frame)")
        by[ev.name][key] += 1
    for name, c in by.items():
        print(f"== {name}: {sum(c.values()) / a.steps:.1f} per step")
        for k, n in c.most_common(15):
            print(f"   {n / a.steps:6.1f}  {k}")


if __name__ == "__main__":
    main()
