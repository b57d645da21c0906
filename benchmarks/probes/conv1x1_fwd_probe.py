"""ResNet-50's stride-1 1x1 convolutions (B=256) on ts_nt_k: forward with the BatchNorm-statistics epilogue and the input
gradient, each timed per shape and compared with the bytes it must move (HBM roofline) and with a device copy of the
same bytes (the achievable bandwidth on this box).

    python benchmarks/probes/conv1x1_fwd_probe.py [--batch 256] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

# (cin, cout, H, count per ResNet-50 step) -- stride-1 1x1 convolutions (conv1, conv3, layer1's downsample)
SHAPES = [(64, 64, 56, 1), (256, 64, 56, 2), (64, 256, 56, 4), (256, 128, 56, 1), (512, 128, 28, 3),
          (128, 512, 28, 4), (512, 256, 28, 1), (1024, 256, 14, 5), (256, 1024, 14, 6), (1024, 512, 14, 1),
          (2048, 512, 7, 2), (512, 2048, 7, 3)]


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    ops = torch.ops.dph
    torch.manual_seed(0)
    from distributed_pytorch_hpc_amd.ops.conv import strided_fwd_geo

    tot = {"fwd": 0.0, "dgrad": 0.0, "copy": 0.0, "convg_fwd": 0.0, "convg_dgrad": 0.0, "best": 0.0}
    for cin, cout, hw, cnt in SHAPES:
        M = a.batch * hw * hw
        x = torch.randn(M, cin, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(cout, cin, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(M, cout, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        src = torch.empty(M * (cin + cout), device="cuda", dtype=torch.bfloat16)
        dst = torch.empty_like(src)
        t_f = _time(lambda: ops.ts_gemm_nt_stats(x, w), a.iters)
        t_d = _time(lambda: ops.ts_gemm_nt(dy, wt), a.iters)
        # the same GEMMs on the LDS-DMA implicit-GEMM kernel (conv3_k GEN) with a one-tap identity geometry
        geo = strided_fwd_geo(hw, hw, 1, 1, 0)
        t_gf = _time(lambda: ops.convg_nt(x, w, geo, True), a.iters)
        t_gd = _time(lambda: ops.convg_nt(dy, wt, geo, False), a.iters)
        t_c = _time(lambda: dst.copy_(src), a.iters) / 2          # read + write of the same byte count
        # the vendor library on the same products (no statistics epilogue): forward X W^T and dgrad dY W
        t_bf = _time(lambda: torch.matmul(x, w.t()), a.iters)
        t_bd = _time(lambda: torch.matmul(dy, w), a.iters)
        gb = M * (cin + cout) * 2 / 1e9
        row = dict(cin=cin, cout=cout, hw=hw, count=cnt, fwd_ms=round(t_f, 4), dgrad_ms=round(t_d, 4),
                   fwd_TBps=round(gb / t_f, 2), dgrad_TBps=round(gb / t_d, 2), copy_TBps=round(gb / t_c, 2),
                   fwd_tflops=round(2 * M * cin * cout / t_f / 1e9, 1), convg_fwd_ms=round(t_gf, 4),
                   convg_dgrad_ms=round(t_gd, 4), blas_fwd_ms=round(t_bf, 4), blas_dgrad_ms=round(t_bd, 4))
        print(json.dumps(row), flush=True)
        tot["fwd"] += cnt * t_f
        tot["dgrad"] += cnt * t_d
        tot["copy"] += cnt * t_c
        tot["convg_fwd"] += cnt * t_gf
        tot["convg_dgrad"] += cnt * t_gd
        tot["best"] += cnt * (min(t_f, t_gf) + min(t_d, t_gd))
        tot["blas_fwd"] = tot.get("blas_fwd", 0.0) + cnt * t_bf
        tot["blas_dgrad"] = tot.get("blas_dgrad", 0.0) + cnt * t_bd
        del x, w, dy, wt, src, dst
    print(json.dumps({k + "_ms_per_step": round(v, 3) for k, v in tot.items()}))


if __name__ == "__main__":
    main()
