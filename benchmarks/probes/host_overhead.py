#!/usr/bin/env python3
"""Is a bench layout's step host-bound?  Builds the workload exactly as bench.py does (one rank, no process group),
then per step measures (a) the host time to ENQUEUE the step (no synchronisation) and (b) the device time between
consecutive steps (CUDA events).  Enqueue ~= device time means the GPU waits on Python; enqueue << device time
means the kernels are the bound.  Optionally dumps a cProfile of a few steps (top functions by own time).

    python benchmarks/probes/host_overhead.py --layout resnet-fsdp --steps 10 --warmup 3 [--cprofile N]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

import bench  # noqa: E402
from distributed_pytorch_hpc_amd.train.bench_layouts import BUILDERS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cprofile", type=int, default=0, help="profile this many steps with cProfile")
    ap.add_argument("--top", type=int, default=35)
    own, rest = ap.parse_known_args()
    args = bench.parse(rest + ["--no-dist"])
    torch.cuda.set_device(0)
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    dev = torch.device("cuda", 0)
    wl = BUILDERS[args.layout](args, 0, 1, dev, lambda m: print(m, file=sys.stderr))
    for i in range(args.warmup):
        wl.step(i)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    enq = []
    for i in range(args.steps):
        ev[i].record()
        t0 = time.perf_counter()
        wl.step(args.warmup + i)
        enq.append(1e3 * (time.perf_counter() - t0))
    ev[-1].record()
    torch.cuda.synchronize()
    dev_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"[host] layout {args.layout}: enqueue median {med(enq):.2f} ms/step, device median {med(dev_ms):.2f} "
          f"ms/step (enqueue/device {med(enq) / med(dev_ms):.2f})")
    print("[host] enqueue ms:", [round(x, 2) for x in enq])
    print("[host] device ms: ", [round(x, 2) for x in dev_ms])
    if own.cprofile:
        pr = cProfile.Profile()
        torch.cuda.synchronize()
        pr.enable()
        for i in range(own.cprofile):
            wl.step(1000 + i)
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(own.top)
        print(s.getvalue())
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(own.top)
        print(s.getvalue())


if __name__ == "__main__":
    main()
