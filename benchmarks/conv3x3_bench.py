#!/usr/bin/env python3
"""Stride-1 3x3 convolutions of ResNet-50 (B=256, bf16, channels-last) and SimpleUNet (B=4, 181 x 360): MIOpen vs the
framework's implicit-GEMM kernels, per pass (forward / input gradient / weight gradient), with TFLOP/s.

    python benchmarks/conv3x3_bench.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, batch, cin, cout, H, W, occurrences per step)
SHAPES = [
    ("resnet50.layer1", 256, 64, 64, 56, 56, 3),
    ("resnet50.layer2", 256, 128, 128, 28, 28, 3),
    ("resnet50.layer3", 256, 256, 256, 14, 14, 5),
    ("resnet50.layer4", 256, 512, 512, 7, 7, 2),
    ("unet.enc1b", 4, 64, 64, 181, 360, 1),
    ("unet.enc2b", 4, 128, 128, 90, 180, 1),
    ("unet.enc3b", 4, 256, 256, 45, 90, 1),
    ("unet.bottleneck_b", 4, 512, 512, 22, 45, 1),
]


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="substring filter on shape names")
    a = ap.parse_args()
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    ops = _lib.ops()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    rows, tot = [], {"miopen": 0.0, "dph": 0.0}
    for name, b, cin, cout, h, w, cnt in SHAPES:
        if a.only and a.only not in name:
            continue
        torch.manual_seed(0)
        x = torch.randn(b, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, 3, 3, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        gy = torch.randn(b, cout, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * b * h * w * cout * cin * 9
        r = {"shape": name, "B": b, "cin": cin, "cout": cout, "H": h, "W": w, "count": cnt}
        # MIOpen
        r["miopen_fwd_ms"] = timeit(lambda: F.conv2d(x, wt, padding=1))
        r["miopen_dgrad_ms"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, wt, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["miopen_wgrad_ms"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, wt, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        # framework kernels (the same calls ops/conv.py's _Conv3x3Fn makes)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        g2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
        wk = wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin).contiguous()
        wf = wt.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, 9 * cout).contiguous()
        gk = torch.empty(cout, 9 * cin, device=dev, dtype=torch.float32)
        r["dph_fwd_ms"] = timeit(lambda: ops.ts_gemm_nt(x2, wk, h, w))
        r["dph_dgrad_ms"] = timeit(lambda: ops.ts_gemm_nt(g2, wf, h, w))
        r["dph_wgrad_ms"] = timeit(lambda: ops.ts_gemm_tn_(gk, g2, x2, False, h, w))
        # parity of the forward against MIOpen (fp32 accumulate both; bf16 output)
        y_ref = F.conv2d(x.float(), wt.float(), padding=1)
        y = ops.ts_gemm_nt(x2, wk, h, w).view(b, h, w, cout).permute(0, 3, 1, 2).float()
        r["fwd_rel_err"] = float((y - y_ref).norm() / y_ref.norm())
        dx_ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), gy.float(), padding=1)
        dx = ops.ts_gemm_nt(g2, wf, h, w).view(b, h, w, cin).permute(0, 3, 1, 2).float()
        r["dgrad_rel_err"] = float((dx - dx_ref).norm() / dx_ref.norm())
        for p in ("fwd", "dgrad", "wgrad"):
            r[f"miopen_{p}_tflops"] = round(flop / r[f"miopen_{p}_ms"] / 1e9, 1)
            r[f"dph_{p}_tflops"] = round(flop / r[f"dph_{p}_ms"] / 1e9, 1)
        m_all = r["miopen_fwd_ms"] + r["miopen_dgrad_ms"] + r["miopen_wgrad_ms"]
        d_all = r["dph_fwd_ms"] + r["dph_dgrad_ms"] + r["dph_wgrad_ms"]
        tot["miopen"] += cnt * m_all
        tot["dph"] += cnt * d_all
        rows.append(r)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    res = {"kernel": "conv3 (LDS-DMA)", "weighted_ms": tot, "shapes": rows}
    print(json.dumps({k: v for k, v in res.items() if k != "shapes"}))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
