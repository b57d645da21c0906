"""Multi-process CPU/gloo test harness (the reference has none: SURVEY.md §4)."""
from __future__ import annotations

import io
import os
import socket
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = fn(rank, world, *args)
        buf = io.BytesIO()
        torch.save(out, buf)   # bytes, not shared-memory tensor handles (the child may exit first)
        q.put((rank, "ok", buf.getvalue()))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_distributed(fn, world: int, *args, timeout: float = 240.0):
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks; returns the per-rank results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            results[rank] = torch.load(io.BytesIO(out), weights_only=True)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
