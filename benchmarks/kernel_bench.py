#!/usr/bin/env python3
"""Per-kernel throughput of the CDNA4 kernels vs the stock PyTorch-ROCm op on Llama-2-7B shapes.

Reports TFLOP/s (attention) or GB/s (memory-bound ops) for both, interleaved in one process
(cdna_hip_programming.md rule 24: A/B from interleaved rounds, median of N).  Random data throughout.

    python benchmarks/kernel_bench.py [--only attn,rmsnorm,...] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd import ops  # noqa: E402
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def bench_attention(B=4, S=4096, H=32, D=128, causal=True):
    dev = "cuda"
    q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    do = torch.randn_like(q)
    scale = 1 / math.sqrt(D)
    flops_fwd = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    o, lse = ops.flash_fwd(q, k, v, scale, causal)
    res = {}
    t = timeit(lambda: ops.flash_fwd(q, k, v, scale, causal))
    res["dph_fwd_ms"], res["dph_fwd_tflops"] = t, flops_fwd / t / 1e9
    t = timeit(lambda: _lib.ops().flash_attn_bwd(do, q, k, v, o, lse, scale, causal))
    res["dph_bwd_ms"], res["dph_bwd_tflops"] = t, 2.5 * flops_fwd / t / 1e9
    qt, kt, vt = (x.transpose(1, 2) for x in (q, k, v))
    t = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
    res["aten_fwd_ms"], res["aten_fwd_tflops"] = t, flops_fwd / t / 1e9
    qg, kg, vg = (x.detach().requires_grad_() for x in (qt, kt, vt))
    out = F.scaled_dot_product_attention(qg, kg, vg, is_causal=causal)
    dot = do.transpose(1, 2)
    t = timeit(lambda: torch.autograd.grad(out, (qg, kg, vg), dot, retain_graph=True))
    res["aten_bwd_ms"], res["aten_bwd_tflops"] = t, 2.5 * flops_fwd / t / 1e9
    return res


def bench_rmsnorm(T=16384, D=4096):
    x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.ones(D, device="cuda", dtype=torch.bfloat16)
    res = {}
    t = timeit(lambda: _lib.ops().rmsnorm_fwd(x, w, 1e-5, None))
    res["dph_fwd_GBps"] = 2 * x.numel() * 2 / t / 1e6
    t = timeit(lambda: _lib.ops().rmsnorm_fwd(x, w, 1e-5, r))
    res["dph_add_fwd_GBps"] = 4 * x.numel() * 2 / t / 1e6
    y, rstd, _ = _lib.ops().rmsnorm_fwd(x, w, 1e-5, None)
    t = timeit(lambda: _lib.ops().rmsnorm_bwd(y, x, w, rstd))
    res["dph_bwd_GBps"] = 3 * x.numel() * 2 / t / 1e6
    t = timeit(lambda: ops.rmsnorm_reference(x, w, 1e-5))
    res["aten_fwd_GBps"] = 2 * x.numel() * 2 / t / 1e6
    return res


def bench_adamw(n=1 << 28):
    p = torch.randn(n, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    g = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: _lib.ops().adamw_step_(p, m, v, g, pb, 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.5, None))
    res = {"dph_GBps": n * 28 / t / 1e6}
    ps = [torch.nn.Parameter(p.clone())]
    ps[0].grad = g.float()
    opt = torch.optim.AdamW(ps, lr=1e-3, fused=True)
    t = timeit(lambda: opt.step())
    res["aten_fused_fp32_GBps"] = n * 32 / t / 1e6
    return res


def bench_swiglu(T=16384, Fh=11008):
    x = torch.randn(T, 2 * Fh, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, Fh, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: _lib.ops().swiglu_fwd(x))
    res = {"dph_fwd_GBps": 3 * T * Fh * 2 / t / 1e6}
    t = timeit(lambda: _lib.ops().swiglu_bwd(dy, x))
    res["dph_bwd_GBps"] = 5 * T * Fh * 2 / t / 1e6
    t = timeit(lambda: ops.swiglu_reference(x))
    res["aten_fwd_GBps"] = 3 * T * Fh * 2 / t / 1e6
    return res


def bench_xent(N=16384, V=32000):
    logits = torch.randn(N, V, device="cuda", dtype=torch.bfloat16)
    tgt = torch.randint(0, V, (N,), device="cuda")
    inv = torch.full((1,), 1.0 / N, device="cuda")
    t = timeit(lambda: _lib.ops().cross_entropy_fwd(logits, tgt, inv, -100, False, 0.0))
    res = {"dph_fwd_GBps": N * V * 2 / t / 1e6}
    t = timeit(lambda: F.cross_entropy(logits.float(), tgt))
    res["aten_fwd_GBps(incl .float())"] = N * V * 2 / t / 1e6
    return res


BENCHES = {"attn": bench_attention, "rmsnorm": bench_rmsnorm, "adamw": bench_adamw, "swiglu": bench_swiglu,
           "xent": bench_xent}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(BENCHES))
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    _lib.require()
    out = {}
    for name in args.only.split(","):
        out[name] = BENCHES[name]()
        print(name, json.dumps({k: round(v, 3) for k, v in out[name].items()}), flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
