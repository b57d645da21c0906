#!/usr/bin/env python3
"""ResNet-50 convolution shapes (B=256, 224^2, bf16, channels-last): MIOpen F.conv2d fwd + bwd vs the same 1x1
convolutions run as plain GEMMs on the NHWC view ([B*H*W, Cin] x [Cin, Cout], hipBLASLt; weight gradient on the
CDNA4 gemm_tn kernel when the channel counts allow).  Prints per-shape ms and the per-step total weighted by how
many times each shape occurs in ResNet-50.

    python benchmarks/conv_bench.py [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, k, stride, H_in, count in ResNet-50)
SHAPES = [
    (64, 64, 1, 1, 56, 1), (256, 64, 1, 1, 56, 2), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3),
    (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
    (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
]


def timeit(fn, iters=10):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from distributed_pytorch_hpc_amd.parallel.linear import _native_wgrad

    torch.backends.cudnn.benchmark = True
    B, dev, dt = a.batch, "cuda", torch.bfloat16
    rows, tot_conv, tot_gemm, tot_dph = [], 0.0, 0.0, 0.0
    for cin, cout, k, s, H, cnt in SHAPES:
        x = torch.randn(B, cin, H, H, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev, dtype=dt) * 0.05).contiguous(memory_format=torch.channels_last)
        Ho = (H + 2 * (k // 2) - k) // s + 1
        gy = torch.randn(B, cout, Ho, Ho, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
        xr, wr = x.detach().requires_grad_(), w.detach().requires_grad_()

        def conv_fb():
            y = F.conv2d(xr, wr, stride=s, padding=k // 2)
            torch.autograd.grad(y, (xr, wr), gy)

        t_conv = timeit(conv_fb)
        row = {"cin": cin, "cout": cout, "k": k, "stride": s, "H": H, "count": cnt, "miopen_fwd_bwd_ms": t_conv}
        tot_conv += cnt * t_conv
        if k == 1:
            xs = x if s == 1 else x[:, :, ::s, ::s]
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, cin)          # NHWC view (copy only when strided)
            w2 = w.reshape(cout, cin)
            g2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            gw = torch.empty(cout, cin, device=dev, dtype=dt)

            def gemm_fb():
                torch.matmul(x2, w2.t())                             # forward
                torch.matmul(g2, w2)                                 # input gradient
                if not _native_wgrad(gw, g2, x2, False):             # weight gradient
                    torch.mm(g2.t(), x2, out=gw)

            t_gemm = timeit(gemm_fb)
            row["gemm_fwd_bwd_ms"] = t_gemm
            tot_gemm += cnt * t_gemm
            if s == 1:   # the framework's CDNA4 tall-skinny kernels (ops.Conv1x1)
                from distributed_pytorch_hpc_amd.ops.conv import _Conv1x1Fn

                def dph_fb():
                    y = _Conv1x1Fn.apply(xr, wr)
                    torch.autograd.grad(y, (xr, wr), gy)

                row["dph_fwd_bwd_ms"] = timeit(dph_fb)
                tot_dph += cnt * row["dph_fwd_bwd_ms"]
            else:
                tot_dph += cnt * t_conv
        else:
            tot_gemm += cnt * t_conv
            if k == 3 and s == 1:   # implicit-GEMM 3x3 kernels (ops.Conv3x3)
                from distributed_pytorch_hpc_amd.ops.conv import _Conv3x3Fn

                def dph3_fb():
                    y = _Conv3x3Fn.apply(xr, wr)
                    torch.autograd.grad(y, (xr, wr), gy)

                row["dph_fwd_bwd_ms"] = timeit(dph3_fb)
                tot_dph += cnt * row["dph_fwd_bwd_ms"]
            else:
                tot_dph += cnt * t_conv
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"batch": B, "resnet50_conv_ms_miopen": tot_conv, "resnet50_conv_ms_1x1_as_gemm": tot_gemm,
           "resnet50_conv_ms_1x1_dph": tot_dph, "shapes": rows}
    print(json.dumps({k: v for k, v in res.items() if k != "shapes"}))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
