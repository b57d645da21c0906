#!/usr/bin/env python3
"""A/B of the wgrad GEMM variants (csrc/gemm.hip: 32 = gemm_tn_k, 8 waves of 128 x 64 on 32x32x16; 16 = gemm_tn16_k on
16x16x32) on the Llama-2-7B weight-gradient shapes, random operands, one
process, interleaved arms (cdna_hip_programming.md rule 24), plus hipBLASLt on the same product with K-contiguous
operands (the layout the library runs fastest; its transposes are not counted) as the target.  Also checks every
variant against an fp32 reference.

    python benchmarks/gemm_mfma_ab.py [--variants 32,128] [--tokens 32768] [--rounds 3] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

SHAPES = {  # name: (M = out features, N = in features)
    "wqkv": (12288, 4096), "wo": (4096, 4096), "w13": (22016, 4096), "w2": (4096, 11008), "output": (32000, 4096),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--variants", default="32,33,16")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    variants = [int(v) for v in a.variants.split(",")]
    _lib.require()
    ops = torch.ops.dph
    K = a.tokens
    res = {}
    # numerics first (small K)
    for shape in variants:
        ops.gemm_tn_mfma_(shape)
        for acc in (False, True):
            ga = torch.randn(1024, 512, device="cuda", dtype=torch.bfloat16)
            xb = torch.randn(1024, 768, device="cuda", dtype=torch.bfloat16)
            c0 = torch.randn(512, 768, device="cuda", dtype=torch.float32)
            c = c0.clone()
            ops.gemm_tn_(c, ga, xb, acc)
            ref = ga.float().t() @ xb.float() + (c0 if acc else 0)
            err = ((c - ref).norm() / ref.norm()).item()
            res[f"relerr_mfma{shape}_acc{int(acc)}"] = err
            assert err < 1e-5, (shape, acc, err)
    for name in a.shapes.split(","):
        M, N = SHAPES[name]
        g = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * K * M * N
        times = {v: [] for v in variants}
        gt, xt = g.t().contiguous(), x.t().contiguous()
        times["blaslt_kcontig"] = []
        for _ in range(a.rounds):
            torch.mm(gt, xt.t(), out=c)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                torch.mm(gt, xt.t(), out=c)
            e.record()
            e.synchronize()
            times["blaslt_kcontig"].append(s.elapsed_time(e) / a.iters)
            for shape in variants:
                ops.gemm_tn_mfma_(shape)
                ops.gemm_tn_(c, g, x, False)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.gemm_tn_(c, g, x, False)
                e.record()
                e.synchronize()
                times[shape].append(s.elapsed_time(e) / a.iters)
        ref = None
        for shape in variants:
            ops.gemm_tn_mfma_(shape)
            ops.gemm_tn_(c, g, x, False)
            if ref is None:
                ref = c.float().clone()
            else:
                res[f"{name}_max_diff_{shape}_vs_{variants[0]}"] = (c.float() - ref).abs().max().item()
        del gt, xt
        row = {f"tflops_mfma{s}": flop / (min(t) * 1e-3) / 1e12 for s, t in times.items()}
        row.update({f"ms_mfma{s}": min(t) for s, t in times.items()})
        res[name] = row
        print(name, json.dumps(row), flush=True)
    ops.gemm_tn_mfma_(0)
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
