#!/usr/bin/env python3
"""Probe: can two RCCL ranks share one MI355X (the only multi-rank RCCL configuration a 1-GPU box offers)?

Spawns 2 processes on cuda:0, creates an nccl (= RCCL) process group and runs an all-reduce, a reduce-scatter, an
all-gather and a send/recv ring with exact known values.  Prints one JSON line per rank; exits non-zero when RCCL
refuses (e.g. "duplicate GPU") or a value is wrong.

    python scripts/probe_rccl_shared_gpu.py [--port 29611]
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    res = {"rank": rank}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        res["all_reduce_ok"] = bool((x == world * (world + 1) / 2).all())
        rs = torch.empty(1 << 19, device="cuda")
        dist.reduce_scatter_tensor(rs, torch.full((world << 19,), 1.0, device="cuda"))
        res["reduce_scatter_ok"] = bool((rs == world).all())
        ag = torch.empty(world << 10, device="cuda")
        dist.all_gather_into_tensor(ag, torch.full((1 << 10,), float(rank), device="cuda"))
        res["all_gather_ok"] = bool(all((ag[r << 10:(r + 1) << 10] == r).all() for r in range(world)))
        send = torch.full((4096,), float(rank), device="cuda")
        recv = torch.empty(4096, device="cuda")
        ops = [dist.P2POp(dist.isend, send, (rank + 1) % world), dist.P2POp(dist.irecv, recv, (rank - 1) % world)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        res["p2p_ok"] = bool((recv == (rank - 1) % world).all())
        torch.cuda.synchronize()
        res["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
        dist.destroy_process_group()
    except Exception as e:  # the refusal is the result
        res["error"] = repr(e)[:500]
    q.put(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=29611)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, a.port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = []
    try:
        out = [q.get(timeout=150) for _ in ps]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    if len(out) < len(ps):
        print(json.dumps({"error": "a rank did not report within 150 s"}), flush=True)
        sys.exit(1)
    ok = True
    for r in sorted(out, key=lambda d: d["rank"]):
        print(json.dumps(r), flush=True)
        ok = ok and "error" not in r and all(v for k, v in r.items() if k.endswith("_ok"))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
