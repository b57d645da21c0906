#!/usr/bin/env python3
"""FP8-GEMM mode vs bf16: loss curves of the same model, data and seed (one GPU).

Data is learnable but synthetic (no datasets here): each sequence follows a fixed random permutation of the vocabulary
with probability 0.9 and jumps to a uniform random token otherwise, so the achievable loss is about
0.1 * ln(V) + H(0.9) ~= 1.4 nats and both runs should get close to it.  Prints one JSON line with both curves.

    python benchmarks/fp8_convergence.py [--model llama2-1b] [--steps 150] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_batch(gen, perm, B, S, V, device):
    t = torch.empty(B, S + 1, dtype=torch.long, device=device)
    t[:, 0] = torch.randint(0, V, (B,), device=device, generator=gen)
    jump = torch.rand(B, S, device=device, generator=gen) < 0.1
    rnd = torch.randint(0, V, (B, S), device=device, generator=gen)
    for i in range(S):
        t[:, i + 1] = torch.where(jump[:, i], rnd[:, i], perm[t[:, i]])
    return t


def run(args, fp8_on: bool):
    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.ops import fp8
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    dev = torch.device("cuda", 0)
    margs = get_preset(args.model, max_seq_len=max(args.seq_len, 256))
    model = build_llama(margs, device=dev, dtype=torch.bfloat16, seed=7)
    if fp8_on:
        fp8.enable_for_llama(model)
    eng = DataParallelEngine(model)
    eng.configure_optimizer(OptimConfig(name="adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    gen = torch.Generator(device=dev).manual_seed(123)
    perm = torch.randperm(margs.vocab_size, device=dev, generator=gen)
    losses = []
    t0 = time.perf_counter()
    try:
        for step in range(args.steps):
            t = make_batch(gen, perm, args.batch, args.seq_len, margs.vocab_size, dev)
            loss = model(t[:, :-1], t[:, 1:])
            loss.backward()
            eng.step()
            eng.zero_grad()
            losses.append(round(float(loss.detach()), 4))
        torch.cuda.synchronize()
    finally:
        fp8.set_fp8(False)
    return losses, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-1b")
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    bf, t_bf = run(args, False)
    f8, t_f8 = run(args, True)
    tail = max(1, args.steps // 10)
    res = {"model": args.model, "steps": args.steps, "tokens_per_step": args.batch * args.seq_len,
           "bf16_losses": bf, "fp8_losses": f8, "bf16_seconds": round(t_bf, 2), "fp8_seconds": round(t_f8, 2),
           "final_mean_bf16": round(sum(bf[-tail:]) / tail, 4), "final_mean_fp8": round(sum(f8[-tail:]) / tail, 4),
           "max_abs_gap": round(max(abs(a - b) for a, b in zip(bf, f8)), 4)}
    print(json.dumps(res), flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh)


if __name__ == "__main__":
    main()
