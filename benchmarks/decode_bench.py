#!/usr/bin/env python3
"""Serving throughput of Llama-2-7B on one MI355X: prefill and decode (KV cache, csrc/decode.hip, HIP-graph steps).

Random-init weights, synthetic prompts (no checkpoints or datasets here).  For each batch size: prefill of
``--prompt`` tokens per sequence (one batched forward), then ``--steps`` decode steps (greedy, the next token
fed back on the device, no host sync inside the timed loop) eager and graph-replayed.  A decode step is
memory-bound: it reads every weight once plus each sequence's cached K/V, so the report includes the effective HBM
rate = (weight bytes + K/V bytes read) / step time, against the MI355X's ~8 TB/s.

    python benchmarks/decode_bench.py [--batches 1 8 32 64] [--prompt 1024] [--steps 64] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 32, 64])
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--modes", nargs="+", choices=["eager", "graph"], default=["eager", "graph"])
    ap.add_argument("--kv-dtype", choices=["bf16", "fp8"], default="bf16",
                    help="KV-cache entries: bf16, or OCP e4m3 (half the cache bytes; opt-in, lossy)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    from distributed_pytorch_hpc_amd.inference import Generator
    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    margs = get_preset(args.model)
    margs = get_preset(args.model, max_seq_len=max(margs.max_seq_len, args.prompt + args.steps + 16))
    model = build_llama(margs, device="cuda", dtype=torch.bfloat16, seed=0)
    wbytes = sum(p.numel() * p.element_size() for p in model.parameters()) - margs.vocab_size * margs.dim * 2
    kv_dtype = torch.float8_e4m3fn if args.kv_dtype == "fp8" else None
    kv_per_tok = margs.n_layers * 2 * margs.kv_heads * margs.head_dim * (1 if kv_dtype is not None else 2)
    rows = []
    for B in args.batches:
        max_len = args.prompt + args.steps + 8
        prompts = torch.randint(0, margs.vocab_size, (B, args.prompt), device="cuda")
        rec = {"batch": B, "prompt": args.prompt, "decode_steps": args.steps}
        for graphs in [m == "graph" for m in args.modes]:
            gen = Generator(model, B, max_len, graphs=graphs, dtype=kv_dtype)
            gen.prefill(prompts)   # warm-up (library heuristics, allocator)
            gen.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            logits = gen.prefill(prompts)
            torch.cuda.synchronize()
            t_prefill = time.perf_counter() - t0
            tok = logits.argmax(-1)
            for _ in range(2):   # eager warm-up step (+ the capture when graphed)
                tok = gen.decode(tok).argmax(-1)
            state = {"tok": tok}

            def step():
                state["tok"] = gen.decode(state["tok"]).argmax(-1)

            dt = timed(step, args.steps)
            avg_len = args.prompt + 2 + args.steps / 2
            bytes_step = wbytes + B * avg_len * kv_per_tok
            key = "graph" if graphs else "eager"
            rec[f"{key}_ms_per_step"] = round(dt * 1e3, 3)
            rec[f"{key}_tokens_per_s"] = round(B / dt, 1)
            rec[f"{key}_hbm_TBps"] = round(bytes_step / dt / 1e12, 2)
            if "prefill_s" not in rec:
                rec["prefill_s"] = round(t_prefill, 3)
                rec["prefill_tokens_per_s"] = round(B * args.prompt / t_prefill, 1)
            del gen
            torch.cuda.empty_cache()
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    res = {"model": args.model, "dtype": "bf16", "kv_cache": args.kv_dtype, "data": "synthetic prompts, random-init weights",
           "weight_bytes": wbytes, "kv_bytes_per_token": kv_per_tok, "rows": rows}
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
