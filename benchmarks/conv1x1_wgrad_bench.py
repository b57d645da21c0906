#!/usr/bin/env python3
"""ResNet-50's stride-1 1x1 weight gradients (B=256, bf16, channels-last): the framework's kernel (``ts_gemm_tn_``:
the LDS-DMA c3w_k form) vs MIOpen, per shape in ms, plus the per-step total weighted by how often each shape occurs.

    python benchmarks/conv1x1_wgrad_bench.py [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, H, count in ResNet-50) -- stride-1 1x1 convolutions
SHAPES = [(64, 64, 56, 1), (256, 64, 56, 2), (64, 256, 56, 4), (256, 128, 56, 1), (512, 128, 28, 3),
          (128, 512, 28, 4), (512, 256, 28, 1), (1024, 256, 14, 5), (256, 1024, 14, 6), (1024, 512, 14, 1),
          (2048, 512, 7, 2), (512, 2048, 7, 3)]


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
    ap.add_argument("--miopen", action="store_true", help="also time MIOpen's weight gradient")
    a = ap.parse_args()
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    torch.backends.cudnn.benchmark = True
    kern = "c3w_k(1x1)"
    rows, tot, tot_mi = [], 0.0, 0.0
    for cin, cout, H, cnt in SHAPES:
        M = a.batch * H * H
        x = torch.randn(M, cin, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, cout, device="cuda", dtype=torch.bfloat16)
        gw = torch.empty(cout, cin, device="cuda", dtype=torch.float32)
        t = timeit(lambda: _lib.ops().ts_gemm_tn_(gw, dy, x, False))
        ref = dy.float().t() @ x.float()
        err = ((gw - ref).norm() / ref.norm()).item()
        r = {"cin": cin, "cout": cout, "H": H, "count": cnt, "ms": t, "tflops": 2 * M * cin * cout / t / 1e9,
             "rel_err": err}
        if a.miopen:
            x4 = x.view(a.batch, H, H, cin).permute(0, 3, 1, 2)
            dy4 = dy.view(a.batch, H, H, cout).permute(0, 3, 1, 2)
            w4 = torch.empty(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16)
            r["miopen_ms"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy4, x4, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
            tot_mi += cnt * r["miopen_ms"]
        tot += cnt * t
        rows.append(r)
        print(f"{cin:5d}->{cout:5d} @{H:3d}  {kern} {t:.3f} ms ({r['tflops']:.0f} TF, err {err:.1e})"
              + (f"  miopen {r['miopen_ms']:.3f}" if a.miopen else ""), flush=True)
    print(f"weighted total per ResNet-50 step: {kern} {tot:.3f} ms" + (f", miopen {tot_mi:.3f} ms" if a.miopen else ""))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"kernel": kern, "rows": rows, "total_ms": tot, "miopen_total_ms": tot_mi}, fh, indent=1)


if __name__ == "__main__":
    main()
