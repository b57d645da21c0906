#!/usr/bin/env python3
"""A/B of the CDNA4 forward / input-gradient GEMM (csrc/gemm_nt.hip) against hipBLASLt (torch.matmul) on the
Llama-2-7B projection shapes at B x S = 32768 tokens, random operands, interleaved arms in one process
(cdna_hip_programming.md rule 24), plus the fused-epilogue variants against their unfused library + kernel chains.

    python benchmarks/gemm_nt_bench.py [--tokens 32768] [--rounds 3] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

# name: (N = out features, K = in features) of y = x W^T; dgrad shapes use W^T ([K, N] -> N' = K, K' = N)
FWD = {"wqkv": (12288, 4096), "wo": (4096, 4096), "w13": (22016, 4096), "w2": (4096, 11008), "output": (32000, 4096)}
DGRAD = {"wqkv.dgrad": (4096, 12288), "wo.dgrad": (4096, 4096), "w13.dgrad": (4096, 22016),
         "w2.dgrad": (11008, 4096), "output.dgrad": (4096, 32000)}
# one tensor-parallel rank's shards at tp = 8 (ragged for the 256 / 64 tile grid)
TP8 = {"wqkv.tp8": (1536, 4096), "w13.tp8": (2752, 4096), "w2.tp8": (4096, 1376), "output.tp8": (4000, 4096),
       "w13.dgrad.tp8": (4096, 2752), "w2.dgrad.tp8": (1376, 4096), "wo.dgrad.tp8": (512, 4096)}


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--shapes", default=",".join(list(FWD) + list(DGRAD)))
    ap.add_argument("--no-fused", action="store_true")
    a = ap.parse_args()
    _lib.require()
    ops = torch.ops.dph
    T = a.tokens
    res = {}
    shapes = {**FWD, **DGRAD, **TP8}
    for name in a.shapes.split(","):
        N, K = shapes[name]
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
        flop = 2.0 * T * N * K
        t = {"blaslt": [], "dph": []}
        ref = x.float() @ w.float().t()
        err = ((ops.gemm_nt(x, w).float() - ref).norm() / ref.norm()).item()
        del ref
        for _ in range(a.rounds):
            t["blaslt"].append(timeit(lambda: torch.matmul(x, w.t()), a.iters))
            t["dph"].append(timeit(lambda: ops.gemm_nt(x, w), a.iters))
        row = {k: {"ms_min": min(v), "ms_med": sorted(v)[len(v) // 2], "tflops_max": flop / min(v) / 1e9}
               for k, v in t.items()}
        row["relerr"] = err
        res[name] = row
        bl, dp = row["blaslt"]["tflops_max"], row["dph"]["tflops_max"]
        print(f"{name:14s} N={N:6d} K={K:6d}  blaslt {bl:7.1f} TF  dph {dp:7.1f} ({dp / bl:.3f})  relerr {err:.2e}",
              flush=True)
        del x, w
    if a.no_fused:
        if a.json:
            with open(a.json, "w") as fh:
                json.dump(res, fh, indent=1)
        return
    # fused epilogues vs library GEMM + separate kernel
    H, D = 11008, 4096
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    w13 = (0.02 * torch.randn(2 * H, D, device="cuda")).to(torch.bfloat16)
    t = {"blaslt+swiglu_fwd": [], "dph_swiglu": []}
    for _ in range(a.rounds):
        t["blaslt+swiglu_fwd"].append(timeit(lambda: ops.swiglu_fwd(torch.matmul(x, w13.t())), a.iters))
        t["dph_swiglu"].append(timeit(lambda: ops.gemm_nt_swiglu(x, w13), a.iters))
    res["w13_fwd_fused"] = {k: min(v) for k, v in t.items()}
    print(f"w13 fwd + SwiGLU: blaslt+kernel {min(t['blaslt+swiglu_fwd']):.3f} ms  fused {min(t['dph_swiglu']):.3f} ms",
          flush=True)
    dy = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    w2t = (0.02 * torch.randn(H, D, device="cuda")).to(torch.bfloat16)
    x13 = torch.randn(T, 2 * H, device="cuda").to(torch.bfloat16)
    t = {"blaslt+swiglu_bwd": [], "dph_dswiglu": []}
    for _ in range(a.rounds):
        t["blaslt+swiglu_bwd"].append(timeit(lambda: ops.swiglu_bwd(torch.matmul(dy, w2t.t()), x13), a.iters))
        t["dph_dswiglu"].append(timeit(lambda: ops.gemm_nt_dswiglu(dy, w2t, x13), a.iters))
    res["w2_dgrad_fused"] = {k: min(v) for k, v in t.items()}
    print(f"w2 dgrad + dSwiGLU: blaslt+kernel {min(t['blaslt+swiglu_bwd']):.3f} ms  fused {min(t['dph_dswiglu']):.3f} ms",
          flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
