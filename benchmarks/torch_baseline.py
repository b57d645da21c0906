#!/usr/bin/env python3
"""Stock PyTorch-ROCm comparator for the headline benchmark (BASELINE.md "How the north-star metric will be
baselined": every config measured once through stock PyTorch-ROCm paths and once through this framework).

Same Llama-2-7B architecture, data and timing protocol as ``bench.py``, but nothing of the framework's runtime:
  * the framework's ops are routed to their ATen equivalents (``F.scaled_dot_product_attention``, eager RMSNorm /
    RoPE / SwiGLU, ``F.cross_entropy``) -- the model code the reference ships (fsdp_tp/llama2_model.py) uses the same
    ATen calls;
  * fp32 parameters, ``torch.autocast(bfloat16)`` compute, ``torch.optim.AdamW`` (``fused=True`` by default,
    ``--adamw foreach`` for the reference's setting, fsdp_tp_example.py:194);
  * N > 1: ``torch.nn.parallel.DistributedDataParallel(device_ids=[local_rank])`` with torch's default 25 MB buckets
    (what the reference's drivers use, e.g. scripts/main.py:257-260).
At B = 8 this stack does not fit 288 GB (fp32 grads + the autocast weight cache + unfused activations), so the default
is B = 4; tokens/s is per-token comparable with bench.py's number.

    python benchmarks/torch_baseline.py [--micro-batch 4] [--steps 4 --warmup 2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 benchmarks/torch_baseline.py --gpus N
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


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--adamw", choices=["fused", "foreach"], default="fused")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--params", choices=["fp32", "bf16"], default="fp32",
                    help="fp32 = fp32 parameters + bf16 autocast (default); bf16 = bf16 parameters, no autocast, "
                         "fused AdamW on the bf16 parameters (its states in bf16: lighter than the framework's fp32 "
                         "master + states, so B = 8 fits)")
    args = ap.parse_args(argv)

    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.runtime import env as rt

    _lib.set_reference_mode(True)   # ATen for every op: nothing of csrc/ runs
    cpu = args.device == "cpu"
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:
        rank, world, local = rt.init_distributed(backend="gloo" if cpu else None, verbose=False)
    else:
        rank, world, local = 0, 1, 0
        if not cpu:
            torch.cuda.set_device(0)
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    margs = get_preset(args.model, max_seq_len=max(args.seq_len, 4096))
    model = build_llama(margs, device=dev, dtype=torch.bfloat16 if args.params == "bf16" else torch.float32,
                        seed=1234)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=None if cpu else [local])
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1,
                            fused=(args.adamw == "fused" and not cpu), foreach=(args.adamw == "foreach"))
    B, S = args.micro_batch, args.seq_len
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    batches = [torch.randint(0, margs.vocab_size, (B, S + 1), device=dev, generator=g) for _ in range(4)]
    amp = torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=args.params == "fp32")

    def step(i):
        t = batches[i % len(batches)]
        with amp:
            loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    def sync_all():
        sync()
        if dist.is_initialized():
            rt.barrier()
        sync()

    for i in range(args.warmup):
        loss = step(i)
    first = float(loss.detach()) if args.warmup else float("nan")
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync_all()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tps = world * B * S * args.steps / elapsed
    if rank == 0:
        rec = {"metric": "tokens/sec, stock PyTorch-ROCm comparator (BASELINE.md)", "value": round(tps, 2),
               "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
               "dtype": "bf16 autocast" if args.params == "fp32" else "bf16",
               "data": "synthetic (random tokens, random-init weights)",
               "config": {"model": "Llama-2-7B" if args.model == "llama2-7b" else args.model,
                          "global_batch": world * B, "seq_len": S,
                          "parallelism": f"torch-ddp{world}" if world > 1 else "single",
                          "optimizer": f"torch.optim.AdamW({args.adamw})", "params": args.params},
               "tokens_per_sec_per_gpu": round(tps / world, 2),
               "peak_hbm_gb": 0.0 if cpu else round(torch.cuda.max_memory_allocated() / 1e9, 2),
               "loss_first_warmup": round(first, 4), "loss_last": round(float(loss.detach()), 4)}
        print(json.dumps(rec), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                json.dump(rec, fh)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
