#!/usr/bin/env python3
"""Per-kernel times of the channels-last 1x1 convolution kernels (csrc/conv1x1.hip) on ResNet-50 shapes (B=256),
with the HBM bytes each must move and the implied fraction of the measured 6.3 TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

SHAPES = [(64, 64, 56), (256, 64, 56), (64, 256, 56), (256, 128, 56), (512, 128, 28), (128, 512, 28),
          (512, 256, 28), (1024, 256, 14), (256, 1024, 14), (1024, 512, 14), (2048, 512, 7), (512, 2048, 7)]


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it


def main():
    _lib.require()
    ops = torch.ops.dph
    out = []
    for cin, cout, H in SHAPES:
        M = 256 * H * H
        x = torch.randn(M, cin, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(cout, cin, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        dy = torch.randn(M, cout, device="cuda", dtype=torch.bfloat16)
        gw = torch.empty(cout, cin, device="cuda", dtype=torch.bfloat16)
        f = t(lambda: ops.ts_gemm_nt(x, w))
        d = t(lambda: ops.ts_gemm_nt(dy, wt))
        g = t(lambda: ops.ts_gemm_tn_(gw, dy, x, False))
        bx, by = M * cin * 2, M * cout * 2
        row = {"cin": cin, "cout": cout, "H": H, "fwd_ms": f, "dgrad_ms": d, "wgrad_ms": g,
               "fwd_bw": (bx + by) / f / 1e9 / 6300, "dgrad_bw": (bx + by) / d / 1e9 / 6300,
               "wgrad_bw": (bx + by) / g / 1e9 / 6300}
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)
        out.append(row)


if __name__ == "__main__":
    main()
