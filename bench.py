#!/usr/bin/env python3
"""Headline benchmark: Llama-2-7B training throughput (tokens/s) on 1..8 MI355X, weak scaling.

Metric and config come from BASELINE.json ("tokens/sec + DDP/FSDP scaling efficiency, Llama-2-7B at
1/2/4/8 MI355X").  Every rank trains the full Llama-2-7B architecture (random init, synthetic tokens)
with a fixed per-GPU batch; N > 1 runs the FSDP engine (reduce-scatter gradients overlapped with
backward, sharded fp32 AdamW state, parameter all-gather overlapped with the next forward) over RCCL.
The timed region holds EXACTLY --steps full optimizer steps (forward + backward + gradient collectives +
AdamW + parameter all-gather), bracketed by a barrier and a device synchronize on both sides; the
reported time is the MAX over ranks; rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

BASELINE_METRIC = "tokens/sec + DDP/FSDP scaling efficiency, Llama-2-7B at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=8,
                    help="sequences per GPU per step (8 x 4096 tokens: ~249 GB peak on one 288 GB MI355X)")
    ap.add_argument("--parallel", choices=["auto", "fsdp", "ddp"], default="auto",
                    help="auto: single-GPU engine for N=1, FSDP (sharded optimizer) for N>1")
    ap.add_argument("--bucket-mb", default="256",
                    help="gradient bucket size in MiB, or 'auto' (alpha-beta fit of comm/cost_model.py, $DPH_COMM_FIT)")
    ap.add_argument("--grad-dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--kernels", choices=["dph", "aten"], default="dph",
                    help="dph: CDNA4 HIP kernels (default); aten: stock PyTorch-ROCm ops (comparator)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--ac", default="none",
                    help="activation checkpointing: none | auto (fit 288 GB) | N (every N-th block)")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the RCCL process group even for one rank (exercises the N>1 collective path)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None,
                    help="process-group backend (default: nccl = RCCL on GPU); gloo lets several ranks share one GPU "
                         "to rehearse the N > 1 path (tests/test_bench_gpu.py)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--fp8", action="store_true",
                    help="opt-in FP8 GEMMs for the projections (ops/fp8.py; e4m3 activations/weights, e5m2 gradients, "
                         "LM head bf16). Reported with dtype 'bf16+fp8-gemm' -- not the bf16 headline number")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: gloo + eager reference ops (tests of the N > 1 code path with tiny models only)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    from distributed_pytorch_hpc_amd.runtime import env as rt

    cpu = args.device == "cpu"
    if world_env > 1 or args.force_dist:
        rank, world, local = rt.init_distributed(backend="gloo" if cpu else args.backend, verbose=not args.quiet)
    else:
        rank, world, local = 0, 1, 0
        if not cpu:
            torch.cuda.set_device(0)
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}", file=sys.stderr)
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel.data_parallel import (DataParallelEngine, MixedPrecision,
                                                                    OptimConfig)

    if not cpu:
        _lib.require()
    if args.kernels == "aten":
        _lib.set_reference_mode(True)
    margs = get_preset(args.model, max_seq_len=max(args.seq_len, 4096))
    dtype = torch.float32 if cpu else torch.bfloat16
    model = build_llama(margs, device=dev, dtype=dtype, seed=1234)
    ac_every = 0
    if args.ac != "none":
        from distributed_pytorch_hpc_amd.parallel.activation_checkpoint import (apply_llama_checkpointing,
                                                                                plan_llama_checkpointing)

        n_par = margs.num_params()
        static_gb = n_par * (4 + (12 / world if world > 1 else 12)) / 1e9
        ac_every = (plan_llama_checkpointing(margs, args.micro_batch, args.seq_len, static_gb=static_gb)
                    if args.ac == "auto" else int(args.ac))
        apply_llama_checkpointing(model, ac_every)
    mode = args.parallel
    if mode == "auto":
        mode = "fsdp" if world > 1 or args.force_dist else "ddp"
    if args.fp8 and not cpu:
        from distributed_pytorch_hpc_amd.ops import fp8 as fp8_mod

        fp8_mod.enable_for_llama(model)
    engine = DataParallelEngine(
        model, shard=(mode == "fsdp"),
        mixed_precision=MixedPrecision(param_dtype=dtype,
                                       reduce_dtype=torch.bfloat16 if args.grad_dtype == "bf16" and not cpu
                                       else torch.float32),
        bucket_cap_mb=args.bucket_mb if args.bucket_mb == "auto" else float(args.bucket_mb))
    engine.configure_optimizer(OptimConfig(name="adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))

    B, S = args.micro_batch, args.seq_len
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    batches = [torch.randint(0, margs.vocab_size, (B, S + 1), device=dev, generator=g) for _ in range(4)]

    def train_step(i):
        t = batches[i % len(batches)]
        loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        engine.step()
        engine.zero_grad()
        return loss

    def sync_all():
        sync()
        if dist.is_initialized():
            rt.barrier()
        sync()

    for i in range(args.warmup):
        loss = train_step(i)
    if args.warmup:
        first_loss = float(loss.detach())
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = train_step(args.warmup + i)
    engine.synchronize()
    sync_all()
    elapsed = time.perf_counter() - t0
    last_loss = float(loss.detach())
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    tokens = world * B * S * args.steps
    tps = tokens / elapsed
    ms = 1000.0 * elapsed / args.steps
    flops_tok = margs.flops_per_token(S)
    mfu = tps / world * flops_tok / 2.5e15
    peak_gb = 0.0 if cpu else torch.cuda.max_memory_allocated() / 1e9
    if rank == 0:
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if cpu else ("bf16+fp8-gemm" if args.fp8 else "bf16"),
            "data": "synthetic (random tokens, random-init weights)",
            "config": {
                "model": "Llama-2-7B" if args.model == "llama2-7b" else args.model,
                "global_batch": world * B,
                "seq_len": S,
                "parallelism": f"{mode}{world}",
                "micro_batch_per_gpu": B,
                "tokens_per_step": world * B * S,
                "kernels": args.kernels,
                "bucket_mb": round(engine.bucket_cap_mb, 1),
                "activation_checkpoint_every": ac_every,
            },
            "tokens_per_sec_per_gpu": round(tps / world, 2),
            "mfu_vs_2.5PF_bf16_dense": round(mfu, 4),
            "peak_hbm_gb": round(peak_gb, 2),
            "loss_first_warmup": round(first_loss, 4) if args.warmup else None,
            "loss_last": round(last_loss, 4),
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if dist.is_initialized():
        rt.cleanup_distributed()


if __name__ == "__main__":
    main()
