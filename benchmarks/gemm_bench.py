#!/usr/bin/env python3
"""Llama-2-7B training GEMM shapes on MI355X: default hipBLASLt selection vs TunableOp-tuned selection.

All GEMMs of a training step (T tokens): forward Y = X W^T, backward dX = dY W, dW = dY^T X, for the fused
wqkv / wo / w13 / w2 / output projections.  ``--tune FILE`` runs PyTorch TunableOp over every shape (tries all
hipBLASLt + rocBLAS solutions) and writes the result table that bench.py loads with ``--tunableop FILE``.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys

import torch


def shapes(T=16384, D=4096, F=11008, V=32000, H=4096 * 3):
    # (name, M, N, K, kind)  kind: nt = X[M,K] @ W[N,K]^T ; nn = dY[M,N'] @ W ; tn = dY^T @ X
    out = []
    for name, n_out, n_in in (("wqkv", H, D), ("wo", D, D), ("w13", 2 * F, D), ("w2", D, F), ("output", V, D)):
        out.append((f"{name}.fwd", T, n_out, n_in, "nt"))
        out.append((f"{name}.dgrad", T, n_in, n_out, "nn"))
        out.append((f"{name}.wgrad", n_out, n_in, T, "tn"))
    return out


def make(kind, M, N, K, dev):
    if kind == "nt":
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        return lambda: torch.matmul(a, b.t())
    if kind == "nn":
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        return lambda: torch.matmul(a, b)
    a = torch.randn(K, M, device=dev, dtype=torch.bfloat16)   # dY [T, M]
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)   # X  [T, N]
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    return lambda: torch.mm(a.t(), b, out=out)


def timeit(fn, iters=20):
    for _ in range(5):
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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--tune", default=None, help="write TunableOp results to this file")
    ap.add_argument("--use", default=None, help="read TunableOp results from this file")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = "cuda"
    if args.tune or args.use:
        import torch.cuda.tunable as tunable

        tunable.enable(True)
        tunable.tuning_enable(bool(args.tune))
        tunable.set_filename(args.tune or args.use)
        if args.tune:
            tunable.set_max_tuning_duration(30)
            tunable.set_max_tuning_iterations(30)
        else:
            tunable.read_file(args.use)
    res = {}
    total_flop, total_ms = 0.0, 0.0
    for name, M, N, K, kind in shapes(args.tokens):
        fn = make(kind, M, N, K, dev)
        ms = timeit(fn)
        tf = 2 * M * N * K / ms / 1e9
        res[name] = {"M": M, "N": N, "K": K, "kind": kind, "ms": round(ms, 4), "tflops": round(tf, 1)}
        total_flop += 2 * M * N * K
        total_ms += ms
        print(f"{name:14s} M={M:6d} N={N:6d} K={K:6d} {kind} {ms:8.3f} ms {tf:7.1f} TF/s", flush=True)
    print(f"TOTAL {total_ms:.2f} ms  {total_flop / total_ms / 1e9:.1f} TF/s (per layer-type set, one each)")
    res["_total"] = {"ms": total_ms, "tflops": total_flop / total_ms / 1e9}
    if args.tune:
        import torch.cuda.tunable as tunable

        tunable.write_file(args.tune)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    sys.exit(main())
