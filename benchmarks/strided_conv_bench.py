#!/usr/bin/env python3
"""ResNet-50's strided convolutions (B=256, bf16, channels-last): MIOpen vs the gathered implicit-GEMM kernels
(ops/conv.py StridedConv2d) per pass -- forward, input gradient (parity classes), weight gradient -- in ms.

    python benchmarks/strided_conv_bench.py [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, k, H_in): stride 2, padding k // 2 -- layer2..4 conv2 (3x3) and downsample (1x1)
SHAPES = [(128, 128, 3, 56), (256, 256, 3, 28), (512, 512, 3, 14),
          (256, 512, 1, 56), (512, 1024, 1, 28), (1024, 2048, 1, 14)]


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
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.ops.conv import (_nhwc2d, strided_dgrad_classes, strided_dgrad_covers_all,
                                                      strided_fwd_geo, strided_out_hw)

    _lib.require()
    ops = _lib.ops()
    torch.backends.cudnn.benchmark = True
    rows = []
    for cin, cout, k, H in SHAPES:
        s, p, B = 2, k // 2, a.batch
        Ho, Wo = strided_out_hw(H, H, k, s, p)
        x = torch.randn(B, cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (0.05 * torch.randn(cout, cin, k, k, device="cuda")).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(B, cout, Ho, Wo, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        mi = {
            "fwd": timeit(lambda: torch.nn.functional.conv2d(x, w, None, s, p)),
            "dgrad": timeit(lambda: conv_bwd(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                             [True, False, False])),
            "wgrad": timeit(lambda: conv_bwd(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                             [False, True, False])),
        }
        x2, dy2 = _nhwc2d(x), _nhwc2d(dy)
        wk = w.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
        geo = strided_fwd_geo(H, H, k, s, p)
        wp = w.permute(1, 2, 3, 0)
        classes = [(g, torch.stack([wp[:, ky, kx, :] for ky, kx in kt], 1).reshape(cin, len(kt) * cout))
                   for g, kt in strided_dgrad_classes(H, H, k, s, p)]
        full = strided_dgrad_covers_all(H, H, k, s, p)

        def dgrad():
            dx2 = (torch.empty if full else torch.zeros)((B * H * H, cin), dtype=torch.bfloat16, device="cuda")
            for g, bk in classes:
                ops.convg_nt_out_(dy2, bk, g, dx2)

        gk = torch.empty(cout, k * k * cin, device="cuda", dtype=torch.float32)

        def wgrad():   # gathered rows for 1x1 and 3x3 alike (ops/conv.py _StridedConvFn)
            ops.convg_tn_(gk, dy2, x2, geo, False)

        ours = {"fwd": timeit(lambda: ops.convg_nt(x2, wk, geo, False)), "dgrad": timeit(dgrad),
                "wgrad": timeit(wgrad)}
        r = {"shape": f"{k}x{k}/2 {cin}->{cout} @{H}", "miopen": mi, "dph": ours}
        rows.append(r)
        print(f"{r['shape']:24s} " + "  ".join(f"{p_}: miopen {mi[p_]:.3f} dph {ours[p_]:.3f} ({mi[p_] / ours[p_]:.2f}x)"
                                              for p_ in ("fwd", "dgrad", "wgrad")), flush=True)
    tot = {w_: sum(r[w_][p_] for r in rows for p_ in ("fwd", "dgrad", "wgrad")) for w_ in ("miopen", "dph")}
    print(f"total ms (one of each): miopen {tot['miopen']:.3f}  dph {tot['dph']:.3f}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"rows": rows, "total": tot}, fh, indent=1)


if __name__ == "__main__":
    main()
