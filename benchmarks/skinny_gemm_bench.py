#!/usr/bin/env python3
"""Decode-sized projections of Llama-2-7B (M = tokens in flight <= 64): the weight-streaming skinny GEMM of
csrc/decode.hip against hipBLASLt (F.linear).  Reports microseconds per call and the weight-read rate (TB/s).

    python benchmarks/skinny_gemm_bench.py [--ms 1 8 32 64] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"wqkv": (12288, 4096), "wo": (4096, 4096), "w13": (22016, 4096), "w2": (4096, 11008), "lm_head": (32000, 4096)}


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=int, nargs="+", default=[1, 2, 8, 16, 32])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.ops.decode import skinny_linear

    _lib.require()
    rows = []
    # several weight copies rotate so the 256 MB MALL does not serve repeated calls from cache
    for name, (n, k) in SHAPES.items():
        ws = [torch.randn(n, k, device="cuda").to(torch.bfloat16) for _ in range(4)]
        for m in args.ms:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            it = {"i": 0}

            def nxt():
                it["i"] = (it["i"] + 1) % len(ws)
                return ws[it["i"]]

            t_s = bench(lambda: skinny_linear(x, nxt()))
            t_b = bench(lambda: F.linear(x, nxt()))
            err = (skinny_linear(x, ws[0]).float() - F.linear(x, ws[0]).float()).abs().max().item()
            byt = n * k * 2
            rec = {"proj": name, "M": m, "N": n, "K": k, "skinny_us": round(t_s, 2), "hipblaslt_us": round(t_b, 2),
                   "skinny_TBps": round(byt / t_s / 1e6, 2), "hipblaslt_TBps": round(byt / t_b / 1e6, 2),
                   "speedup": round(t_b / t_s, 2), "max_abs_diff": err}
            rows.append(rec)
            print(json.dumps(rec), flush=True)
        del ws
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
