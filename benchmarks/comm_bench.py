#!/usr/bin/env python3
"""Collective microbenchmark over RCCL (xGMI) or gloo: broadcast, all-reduce, all-gather, reduce-scatter,
all-to-all and point-to-point send/recv, with algorithm and bus bandwidth in GB/s (1e9 bytes).

Capability parity with tests/torch_comm_bench.py and tests/all_reduce_test.py of the reference (broadcast +
all-reduce timing over 10^3..10^8 fp32 elements, CSV with an environment header) with its defects fixed (X11):
  * bandwidth in GB/s with 1e9 (the reference divides by 1024^3 and labels it GB/s);
  * device-side timing with HIP events over ``--iters`` back-to-back ops, barrier OUTSIDE the timed window;
  * ``--sizes`` is honoured; all six collective families; bus-bandwidth factors as in rccl-tests
    (all-reduce 2(n-1)/n, all-gather / reduce-scatter / all-to-all (n-1)/n, broadcast and p2p 1).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/comm_bench.py \
        --ops all_reduce,all_gather --sizes 1e3,1e6,1e8 --csv results/comm.csv
    (gloo on CPU: add --backend gloo)
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402

BUSBW = {"all_reduce": lambda n: 2 * (n - 1) / n, "custom_all_reduce": lambda n: 2 * (n - 1) / n, "all_gather": lambda n: (n - 1) / n,
         "reduce_scatter": lambda n: (n - 1) / n, "all_to_all": lambda n: (n - 1) / n,
         "broadcast": lambda n: 1.0, "send_recv": lambda n: 1.0}


_CAR = {}


def _custom(world):
    """XgmiAllReduce over the world group (comm/custom_allreduce.py), created once."""
    if "car" not in _CAR:
        from distributed_pytorch_hpc_amd.comm.custom_allreduce import XgmiAllReduce

        _CAR["car"] = XgmiAllReduce(None, max_bytes=int(os.environ.get("CAR_MAX_BYTES", str(64 << 20))),
                                    max_blocks=int(os.environ.get("CAR_BLOCKS", "64")))
    return _CAR["car"]


def run_op(op, x, out, world, rank, group=None):
    if op == "all_reduce":
        dist.all_reduce(x, group=group)
    elif op == "custom_all_reduce":   # direct peer reads over xGMI (one-shot / two-shot), in place
        _custom(world).all_reduce(x)
    elif op == "broadcast":
        dist.broadcast(x, src=0, group=group)
    elif op == "all_gather":
        dist.all_gather_into_tensor(out, x, group=group)
    elif op == "reduce_scatter":
        dist.reduce_scatter_tensor(out, x, group=group)
    elif op == "all_to_all":
        dist.all_to_all_single(out, x, group=group)
    elif op == "send_recv":   # ring shift: every rank sends to rank+1 and receives from rank-1
        ops = [dist.P2POp(dist.isend, x, (rank + 1) % world), dist.P2POp(dist.irecv, out, (rank - 1) % world)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def bench_one(op, numel, dtype, device, iters, warmup):
    world, rank = dist.get_world_size(), dist.get_rank()
    numel = max(world, numel // world * world)
    if op == "custom_all_reduce":
        if device.type != "cuda":
            return None
        numel = max(8, numel // 8 * 8)
        if numel * torch.empty((), dtype=dtype).element_size() > _custom(world).max_bytes:
            return None
    x = torch.ones(numel, dtype=dtype, device=device)
    if op == "all_gather":
        out = torch.empty(numel * world, dtype=dtype, device=device)
    elif op == "reduce_scatter":
        out = torch.empty(numel // world, dtype=dtype, device=device)
    else:
        out = torch.empty_like(x)
    for _ in range(warmup):
        run_op(op, x, out, world, rank)
    rt.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            run_op(op, x, out, world, rank)
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 1e3 / iters
    else:
        t0 = time.perf_counter()
        for _ in range(iters):
            run_op(op, x, out, world, rank)
        t = (time.perf_counter() - t0) / iters
    tt = torch.tensor([t], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = tt.item()
    # message size as in rccl-tests: all-gather counts the gathered output, every other op its input
    nbytes = numel * x.element_size() * (world if op == "all_gather" else 1)
    algbw = nbytes / t / 1e9
    return {"op": op, "numel": numel, "bytes": nbytes, "dtype": str(dtype).replace("torch.", ""), "world": world,
            "time_us": t * 1e6, "algbw_GBps": algbw, "busbw_GBps": algbw * BUSBW[op](world)}


def env_header() -> dict:
    h = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None), "backend": dist.get_backend(),
         "world": dist.get_world_size(), "host": rt.hostname()}
    if torch.cuda.is_available():
        h["gpu"] = torch.cuda.get_device_name(0)
        try:
            h["rccl"] = ".".join(map(str, torch.cuda.nccl.version()))
        except Exception:
            pass
    for k in sorted(os.environ):
        if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_")):
            h[k] = os.environ[k]
    return h


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ops", default="broadcast,all_reduce,all_gather,reduce_scatter,all_to_all,send_recv",
                    help="comma list; 'custom_all_reduce' adds the direct-peer-read xGMI all-reduce (GPU only)")
    ap.add_argument("--sizes", default="1e3,1e4,1e5,1e6,1e7,1e8", help="elements per rank (comma list)")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--fit", default=None,
                    help="write per-op alpha-beta fits (comm/cost_model.py) here; DPH_COMM_FIT=<file> makes the "
                         "data-parallel engine size its buckets from them (bucket_cap_mb='auto')")
    args = ap.parse_args(argv)
    rank, world, local = rt.init_distributed(backend=args.backend, verbose=False)
    device = rt.device_for(local, dist.get_backend())
    dtype = getattr(torch, args.dtype)
    rows = []
    for op in args.ops.split(","):
        for s in args.sizes.split(","):
            r = bench_one(op, int(float(s)), dtype, device, args.iters, args.warmup)
            if r is None:   # custom all-reduce: CPU run or message above its staging buffer
                continue
            rows.append(r)
            if rank == 0:
                print(f"{op:15s} {r['bytes'] / 1e6:11.3f} MB  {r['time_us']:11.1f} us  algbw {r['algbw_GBps']:8.2f} GB/s"
                      f"  busbw {r['busbw_GBps']:8.2f} GB/s", flush=True)
    if rank == 0:
        if args.csv:
            os.makedirs(os.path.dirname(os.path.abspath(args.csv)), exist_ok=True)
            with open(args.csv, "w", newline="") as fh:
                for k, v in env_header().items():
                    fh.write(f"# {k}: {v}\n")
                w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
        if args.json:
            with open(args.json, "w") as fh:
                json.dump({"env": env_header(), "results": rows}, fh, indent=1)
        if args.fit:
            from distributed_pytorch_hpc_amd.comm.cost_model import BUS_FACTOR, fit_alpha_beta, save_fits

            fits = {}
            for op in {r["op"] for r in rows}:
                if op not in BUS_FACTOR:
                    continue
                samples = [(r["bytes"], r["time_us"] * 1e-6) for r in rows if r["op"] == op]
                if len(samples) >= 2:
                    fits[op] = fit_alpha_beta(op, world, samples)
                    print(f"fit {op:15s} alpha {fits[op].alpha_s * 1e6:9.2f} us  "
                          f"beta_bus {fits[op].beta_bus_Bps / 1e9:9.2f} GB/s", flush=True)
            save_fits(fits, args.fit)
    rt.cleanup_distributed()


if __name__ == "__main__":
    main()
