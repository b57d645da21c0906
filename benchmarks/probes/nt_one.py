#!/usr/bin/env python3
"""Run one forward / input-gradient GEMM shape (C = A B^T, K-contiguous operands) a few times on the CDNA4 NT kernel
or hipBLASLt, for rocprofv3 counter collection (cdna_hip_programming.md §7)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--n", type=int, default=12288)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--hipblaslt", action="store_true")
    ap.add_argument("--variant", type=int, default=0, help="plain-store GEMM form: 0 = gemm_nt_k, 6 = gemm_nt4_k")
    a = ap.parse_args()
    _lib.require()
    torch.ops.dph.gemm_nt_variant(a.variant)
    x = torch.randn(a.m, a.k, device="cuda").to(torch.bfloat16)
    w = (0.02 * torch.randn(a.n, a.k, device="cuda")).to(torch.bfloat16)
    for _ in range(a.iters):
        if a.hipblaslt:
            torch.matmul(x, w.t())
        else:
            torch.ops.dph.gemm_nt(x, w)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
