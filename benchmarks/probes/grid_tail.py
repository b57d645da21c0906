#!/usr/bin/env python3
"""Grid-tail probe: time per 128-row tile of the 1x1 (ts_gemm_nt) and stride-1 3x3 (conv3_k via ts_gemm_nt with H, W)
forward kernels as the row count crosses a multiple of the resident workgroup slots.  If a launch whose grid just
exceeds k full rounds costs about a whole extra round, the per-tile time jumps there -- the tail the weight-gradient
kernel's split-K rounding had (profiles/r4/c3w_rounds/).  Prints one JSON line per (kernel, N, K, row tiles)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    _lib.require()
    ops = _lib.ops()
    # (kind, N, K): ResNet-50 1x1 shapes at 14 x 14 / 7 x 7 and a 3x3 at 14 x 14
    cases = [("1x1", 256, 1024), ("1x1", 1024, 256), ("1x1", 512, 2048), ("1x1", 2048, 512), ("3x3", 256, 256)]
    for kind, N, K in cases:
        for tiles in (96, 128, 160, 192, 256, 320, 384, 392, 400, 448, 512, 520, 576, 640, 768, 784, 800):
            M = tiles * 128
            if kind == "3x3":
                H = W = 16   # M = tiles * 128 rows = (tiles / 2) images of 16 x 16
                if M % (H * W):
                    continue
            a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            if kind == "1x1":
                b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
                t = timeit(lambda: ops.ts_gemm_nt(a, b))
            else:
                b = torch.randn(N, 9 * K, device="cuda", dtype=torch.bfloat16)
                t = timeit(lambda: ops.ts_gemm_nt(a, b, H, W))
            print(json.dumps({"kind": kind, "N": N, "K": K, "row_tiles": tiles, "ms": round(t, 4),
                              "us_per_row_tile": round(1000 * t / tiles, 3)}), flush=True)


if __name__ == "__main__":
    main()
