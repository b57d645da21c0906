#!/usr/bin/env python3
"""One weight-gradient GEMM shape (dW[N, K] = dY^T X over 32768 tokens) on the framework's CDNA4 kernel, looped --iters
times: the target of a rocprofv3 --pmc pass or an s_memtime-free timing.

    python benchmarks/probes/wgrad_one.py [--shape w13] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

SHAPES = {"wqkv": (12288, 4096), "wo": (4096, 4096), "w13": (22016, 4096), "w2": (4096, 11008),
          "output": (32000, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="w13")
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _lib.require()
    N, K = SHAPES[a.shape]
    dy = torch.randn(a.tokens, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(a.tokens, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.ops.dph.gemm_tn_(c, dy, x, False)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        torch.ops.dph.gemm_tn_(c, dy, x, False)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / a.iters
    print(f"{a.shape}: {ms:.3f} ms  {2.0 * a.tokens * N * K / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
