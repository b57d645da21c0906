#!/usr/bin/env python3
"""Per-kernel times of the channels-last 1x1 / 3x3 convolution kernels (csrc/conv1x1.hip) on ResNet-50 shapes
(B=256), next to MIOpen's time for the same direction (forward, input gradient, weight gradient), with the HBM
bytes each must move and the implied fraction of the measured 6.3 TB/s (1x1) or the TFLOP/s (3x3)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

SHAPES3 = [(64, 56), (128, 28), (256, 14), (512, 7)]
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


def miopen_parts(x4, w4, gy4, pad):
    """MIOpen forward / input-gradient / weight-gradient times of one convolution (channels-last bf16)."""
    conv = torch.ops.aten.convolution_backward
    f = t(lambda: torch.nn.functional.conv2d(x4, w4, padding=pad))
    d = t(lambda: conv(gy4, x4, w4, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False]))
    g = t(lambda: conv(gy4, x4, w4, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False]))
    return f, d, g


def cl(t4):
    return t4.contiguous(memory_format=torch.channels_last)


def main():
    _lib.require()
    torch.backends.cudnn.benchmark = True
    ops = torch.ops.dph
    out = []
    for c, H in SHAPES3:
        M = 256 * H * H
        x4 = cl(torch.randn(256, c, H, H, device="cuda", dtype=torch.bfloat16))
        w4 = cl(torch.randn(c, c, 3, 3, device="cuda", dtype=torch.bfloat16) * 0.05)
        gy4 = cl(torch.randn(256, c, H, H, device="cuda", dtype=torch.bfloat16))
        x, dy = x4.permute(0, 2, 3, 1).reshape(M, c), gy4.permute(0, 2, 3, 1).reshape(M, c)
        wk = w4.permute(0, 2, 3, 1).reshape(c, 9 * c).contiguous()
        wf = w4.flip(2, 3).permute(1, 2, 3, 0).reshape(c, 9 * c).contiguous()
        gk = torch.empty(c, 9 * c, device="cuda", dtype=torch.bfloat16)
        f = t(lambda: ops.ts_gemm_nt(x, wk, H, H))
        d = t(lambda: ops.ts_gemm_nt(dy, wf, H, H))
        g = t(lambda: ops.ts_gemm_tn_(gk, dy, x, False, H, H))
        mf, md, mg = miopen_parts(x4, w4, gy4, 1)
        tf = 2.0 * M * c * 9 * c / 1e9
        row = {"k": 3, "c": c, "H": H, "fwd_ms": f, "dgrad_ms": d, "wgrad_ms": g, "miopen_fwd_ms": mf,
               "miopen_dgrad_ms": md, "miopen_wgrad_ms": mg, "fwd_tflops": tf / f, "dgrad_tflops": tf / d,
               "wgrad_tflops": tf / g}
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)
        out.append(row)
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
        mf, md, mg = miopen_parts(cl(x.view(256, H, H, cin).permute(0, 3, 1, 2)), cl(w.view(cout, cin, 1, 1)),
                                  cl(dy.view(256, H, H, cout).permute(0, 3, 1, 2)), 0)
        frac = lambda ms: (bx + by) / (ms * 1e-3) / 6.3e12   # noqa: E731
        row = {"k": 1, "cin": cin, "cout": cout, "H": H, "fwd_ms": f, "dgrad_ms": d, "wgrad_ms": g,
               "miopen_fwd_ms": mf, "miopen_dgrad_ms": md, "miopen_wgrad_ms": mg,
               "fwd_bw": frac(f), "dgrad_bw": frac(d), "wgrad_bw": frac(g)}
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)
        out.append(row)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
