#!/usr/bin/env python3
"""Run one weight-gradient GEMM shape a few times (for rocprofv3 counter collection)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=22016)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--hipblaslt", action="store_true")
    a = ap.parse_args()
    _lib.require()
    g = torch.randn(a.k, a.m, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(a.k, a.n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.iters):
        if a.hipblaslt:
            torch.mm(g.t(), x, out=c)
        else:
            torch.ops.dph.gemm_tn_(c, g, x, False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
