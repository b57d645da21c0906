#!/usr/bin/env python3
"""Point-to-point bandwidth: rank-0 fan-out (the reference's tests/send_recv_test.py: rank 0 sends a 40 MB fp32
tensor to every other rank) plus the full pairwise matrix (every src -> dst pair, one pair at a time), which on an
MI355X node measures each direct xGMI link.  Also the 1-element smoke test of tests/test_torchrun.py (--smoke).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/send_recv_test.py [--matrix]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def fanout(t, dev, iters):
    rank, world = dist.get_rank(), dist.get_world_size()
    times = []
    for it in range(iters + 2):
        rt.barrier()
        _sync(dev)
        t0 = time.perf_counter()
        if rank == 0:
            for d in range(1, world):
                dist.send(t, d)
        else:
            dist.recv(t, 0)
        _sync(dev)
        if it >= 2:
            times.append(time.perf_counter() - t0)
    return sum(times) / len(times)


def matrix(t, dev, iters):
    rank, world = dist.get_rank(), dist.get_world_size()
    bw = [[0.0] * world for _ in range(world)]
    for s in range(world):
        for d in range(world):
            if s == d:
                continue
            rt.barrier()
            if rank in (s, d):
                for it in range(iters + 2):
                    if it == 2:
                        _sync(dev)
                        t0 = time.perf_counter()
                    if rank == s:
                        dist.send(t, d)
                    else:
                        dist.recv(t, s)
                _sync(dev)
                el = (time.perf_counter() - t0) / iters
                if rank == s:
                    bw[s][d] = t.numel() * t.element_size() / el / 1e9
    out = torch.tensor(bw, dtype=torch.float64, device=dev)
    dist.all_reduce(out)
    return out.tolist()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=10000 * 1000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--matrix", action="store_true")
    ap.add_argument("--smoke", action="store_true", help="1-element rank0 -> all send/recv check")
    ap.add_argument("--backend", default=None)
    ap.add_argument("--json", default=None)
    args = ap.parse_args(argv)
    rank, world, local = rt.init_distributed(backend=args.backend, verbose=False)
    dev = rt.device_for(local, dist.get_backend())
    res = {"world": world, "backend": dist.get_backend()}
    if args.smoke:
        t = torch.tensor([float(rank)], device=dev)
        if rank == 0:
            for d in range(1, world):
                dist.send(torch.tensor([42.0], device=dev), d)
        else:
            dist.recv(t, 0)
            assert t.item() == 42.0
        res["smoke"] = "ok"
    t = torch.zeros(args.numel, device=dev)
    res["fanout_s"] = fanout(t, dev, args.iters)
    res["fanout_GBps_per_peer"] = t.numel() * 4 * (world - 1) / res["fanout_s"] / 1e9
    if args.matrix:
        res["matrix_GBps"] = matrix(t, dev, args.iters)
    if rank == 0:
        print(json.dumps(res, indent=1))
        if args.json:
            with open(args.json, "w") as fh:
                json.dump(res, fh, indent=1)
    rt.cleanup_distributed()


if __name__ == "__main__":
    main()
