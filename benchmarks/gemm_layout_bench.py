#!/usr/bin/env python3
"""Weight-storage layout study for the Llama-2-7B training GEMMs on MI355X (hipBLASLt).

Every linear layer needs three GEMMs per step (T tokens): forward Y = X W^T, input gradient dX = dY W and weight
gradient dW = dY^T X.  hipBLASLt picks different kernels for each operand-transposition pattern, so the storage
layout of W decides which three patterns run:

  A ("out_in", nn.Linear):  W stored [out, in]      fwd mm(X, W.t())   dgrad mm(dY, W)      wgrad mm(dY.t(), X) -> [out, in]
  B ("in_out", transposed): W^T stored [in, out]    fwd mm(X, Wt)      dgrad mm(dY, Wt.t()) wgrad mm(X.t(), dY) -> [in, out]

Prints per-shape times / TFLOP/s for both layouts and the per-step total; JSON with --json.
"""
from __future__ import annotations

import argparse
import json
import statistics

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def layers(D=4096, F=11008, V=32000):
    return [("wqkv", 3 * D, D), ("wo", D, D), ("w13", 2 * F, D), ("w2", D, F), ("output", V, D)]


def timeit(fn, iters=15):
    for _ in range(4):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda")
    _lib.require()
    T = args.tokens
    out = {}
    tot = {}
    for name, n_out, n_in in layers():
        x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        gy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n_out, n_in, device=dev, dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        gw_a = torch.empty(n_out, n_in, device=dev, dtype=torch.bfloat16)
        gw_b = torch.empty(n_in, n_out, device=dev, dtype=torch.bfloat16)
        gyt = gy.t().contiguous()
        xt = x.t().contiguous()
        flop = 2.0 * T * n_in * n_out
        cases = {
            "A.fwd": lambda: torch.mm(x, w.t()),
            "A.dgrad": lambda: torch.mm(gy, w),
            "A.wgrad": lambda: torch.mm(gy.t(), x, out=gw_a),
            "B.fwd": lambda: torch.mm(x, wt),
            "B.dgrad": lambda: torch.mm(gy, wt.t()),
            "B.wgrad": lambda: torch.mm(x.t(), gy, out=gw_b),
            # C: weight gradient from K-contiguous (transposed) operand copies: dW = (dY^T) (X^T)^T
            "C.wgrad": lambda: torch.mm(gyt, xt.t(), out=gw_a),
            "C.transpose_dy": lambda: gyt.copy_(gy.t()),
            "C.transpose_x": lambda: xt.copy_(x.t()),
            # D: the framework's CDNA4 weight-gradient kernel on the token-major operands (csrc/gemm.hip)
            "D.wgrad": lambda: torch.ops.dph.gemm_tn_(gw_a, gy, x, False),
            # E: input gradient through a HIP-transposed weight (parallel/linear.py _dgrad)
            "E.dgrad": lambda: torch.mm(gy, torch.ops.dph.transpose2d(w).t()),
            "E.transpose_w": lambda: torch.ops.dph.transpose2d(w),
        }
        for k, fn in cases.items():
            ms = timeit(fn)
            out[f"{name}.{k}"] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
            tot[k[0]] = tot.get(k[0], 0.0) + ms * (1 if name == "output" else 32)
            print(f"{name:7s} {k:8s} {ms:8.3f} ms {flop / ms / 1e9:8.1f} TF", flush=True)
        del x, gy, w, wt, gw_a, gw_b, gyt, xt
        torch.cuda.empty_cache()
    out["per_step_ms"] = {k: round(v, 2) for k, v in tot.items()}
    print("per-step GEMM time (32 layers + output):", out["per_step_ms"], flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
