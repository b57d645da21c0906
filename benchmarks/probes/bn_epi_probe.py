"""BatchNorm backward reduction: own pass vs the consumer convolution's dgrad epilogue, on ResNet-50's B=256 shapes.

For each bottleneck stage and each BatchNorm whose dy a convolution dgrad produces (bn2 <- conv3 1x1, bn1 <- conv2 3x3,
the previous bn3 <- conv1 1x1 + residual add) this times, with CUDA events over ``--iters`` calls:
  unfused: ts_gemm_nt (+ add)        + bn_act_bwd (its reduction pass + finalize + dx pass)
  fused:   ts_gemm_nt_bnred (+ add)  + bn_act_bwd(pre_part=...) (finalize + dx pass)
and prints per-shape ms and the saving.  Synthetic bf16 data; numerics are covered by tests/test_bn_epilogue_gpu.py.

    python benchmarks/probes/bn_epi_probe.py [--batch 256] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


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
    dev = "cuda"
    torch.manual_seed(0)
    rows = []
    for hw, w in ((56, 64), (28, 128), (14, 256), (7, 512)):
        M = a.batch * hw * hw
        for kind in ("bn2<-conv3", "bn1<-conv2", "bn3<-conv1"):
            if kind == "bn2<-conv3":
                C, K, H, W = w, 4 * w, 0, 0
            elif kind == "bn1<-conv2":
                C, K, H, W = w, w, hw, hw
            else:
                C, K, H, W = 4 * w, w, 0, 0
            A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            B = (torch.randn(C, 9 * K if H else K, device=dev) * 0.05).to(torch.bfloat16)
            x = torch.randn(a.batch, C, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            res = torch.randn_like(x) if kind == "bn3<-conv1" else None
            add = torch.randn(M, C, device=dev, dtype=torch.bfloat16) if res is not None else None
            wt = torch.ones(C, device=dev, dtype=torch.bfloat16)
            bs = torch.zeros(C, device=dev, dtype=torch.bfloat16)
            bits = torch.empty(M * C // 8, device=dev, dtype=torch.uint8) if res is not None else None
            _, mean, invstd, ss = ops.bn_act_fwd(x, res, wt, bs, None, None, 0.1, 1e-5, True, None, None, bits)
            ssx = None if res is not None else ss

            def unfused():
                dy = ops.ts_gemm_nt(A, B, H, W, add)
                return ops.bn_act_bwd(dy.view(x.shape[0], hw, hw, C).permute(0, 3, 1, 2), x, x, mean, invstd, wt,
                                      True, res is not None, True, ssx, None, None, bits)

            def fused():
                dy, part = ops.ts_gemm_nt_bnred(A, B, H, W, add, 0, x, mean, invstd, ssx, bits)
                return ops.bn_act_bwd(dy.view(x.shape[0], hw, hw, C).permute(0, 3, 1, 2), x, x, mean, invstd, wt,
                                      True, res is not None, True, ssx, None, None, bits, part)

            def gemm():
                return ops.ts_gemm_nt(A, B, H, W, add)

            def gemm_red():
                return ops.ts_gemm_nt_bnred(A, B, H, W, add, 0, x, mean, invstd, ssx, bits)

            t = {n: _time(f, a.iters) for n, f in (("unfused", unfused), ("fused", fused), ("gemm", gemm),
                                                    ("gemm_bnred", gemm_red))}
            row = dict(hw=hw, C=C, K=K, kind=kind, **{k: round(v, 4) for k, v in t.items()})
            row["saved_ms"] = round(t["unfused"] - t["fused"], 4)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del A, B, x, res, add, bits
    tot_u = sum(r["unfused"] for r in rows)
    tot_f = sum(r["fused"] for r in rows)
    print(json.dumps({"total_unfused_ms": round(tot_u, 3), "total_fused_ms": round(tot_f, 3),
                      "epilogue_cost_ms": round(sum(r["gemm_bnred"] - r["gemm"] for r in rows), 3)}))


if __name__ == "__main__":
    main()
