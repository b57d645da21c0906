#!/usr/bin/env python3
"""Broadcast + all-reduce latency/bandwidth sweep, appended to a results log.

Capability parity with the reference's tests/all_reduce_test.py:1-177 (broadcast and all-reduce of 10^3..10^8 fp32
elements, 2 warm-up + 20 timed runs, one line per op/size appended to ``benchmark_results.log``), with its defects
fixed: ``--tensor-sizes`` is honoured instead of being overwritten, each op is timed per call
with device events (no barrier inside the timed window), and bandwidth is GB/s with 10^9 bytes (algbw = bytes / t,
busbw = algbw x 2(n-1)/n for all-reduce, x 1 for broadcast).  The broader sweep (all-gather, reduce-scatter,
all-to-all, send/recv, custom xGMI all-reduce, CSV/JSON) is benchmarks/comm_bench.py.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/all_reduce_test.py
    ... --backend gloo --tensor-sizes 1e3,1e5      (CPU)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402


def _timed(fn, dev) -> float:
    if dev.type == "cuda":
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / 1e3
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def run(sizes, warmup: int, iters: int, dev, dtype) -> list[dict]:
    rank, world = dist.get_rank(), dist.get_world_size()
    rows = []
    for n in sizes:
        x = torch.ones(n, dtype=dtype, device=dev)
        nbytes = n * x.element_size()
        for op in ("broadcast", "all_reduce"):
            fn = (lambda: dist.broadcast(x, src=0)) if op == "broadcast" else (lambda: dist.all_reduce(x))
            for _ in range(warmup):
                fn()
            rt.barrier()
            ts = [_timed(fn, dev) for _ in range(iters)]
            # the slowest rank defines the collective's time
            t = torch.tensor(ts, dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ts = t.tolist()
            mean = statistics.fmean(ts)
            factor = 2 * (world - 1) / world if op == "all_reduce" else 1.0
            rows.append({"op": op, "numel": n, "bytes": nbytes, "world": world, "mean_s": mean,
                         "std_s": statistics.pstdev(ts), "min_s": min(ts), "max_s": max(ts),
                         "algbw_GBps": nbytes / mean / 1e9, "busbw_GBps": nbytes / mean / 1e9 * factor})
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--tensor-sizes", "--tensor_sizes", default="1e3,1e4,1e5,1e6,1e7,1e8",
                    help="elements per rank, comma list (honoured, unlike the reference)")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--backend", default=None, help="nccl (RCCL) on GPU, gloo on CPU (default: by device)")
    ap.add_argument("--log-file", default="results/benchmark_results.log")
    ap.add_argument("--json", default=None)
    args = ap.parse_args(argv)
    rank, world, local = rt.init_distributed(backend=args.backend, verbose=False)
    backend = dist.get_backend()
    dev = rt.device_for(local, backend)
    sizes = [int(float(s)) for s in args.tensor_sizes.split(",") if s]
    rows = run(sizes, args.warmup, args.iters, dev, getattr(torch, args.dtype))
    if rank == 0:
        ver = None
        if backend == "nccl":
            try:
                ver = ".".join(map(str, torch.cuda.nccl.version()))
            except Exception:
                pass
        os.makedirs(os.path.dirname(os.path.abspath(args.log_file)), exist_ok=True)
        with open(args.log_file, "a") as fh:
            for r in rows:
                line = (f"{backend} {ver or ''} world={world} {r['op']} numel={r['numel']} bytes={r['bytes']}: "
                        f"mean {r['mean_s']:.6e} s min {r['min_s']:.6e} s max {r['max_s']:.6e} s "
                        f"algbw {r['algbw_GBps']:.3f} GB/s busbw {r['busbw_GBps']:.3f} GB/s")
                fh.write(line + "\n")
                print(line, flush=True)
        if args.json:
            with open(args.json, "w") as fh:
                json.dump({"backend": backend, "rccl": ver, "rows": rows}, fh, indent=1)
        print(json.dumps({"benchmark": "all_reduce_test", "backend": backend, "world": world,
                          "sizes": sizes, "n_rows": len(rows)}), flush=True)
    rt.cleanup_distributed()


if __name__ == "__main__":
    main()
