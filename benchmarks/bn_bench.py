#!/usr/bin/env python3
"""Bandwidth of the fused BatchNorm(+residual)+ReLU kernels (csrc/batchnorm.hip) at every ResNet-50 BN shape of a
B = 256, 224 x 224 channels-last bf16 step, against a device copy of the same activation.

Traffic counted per call (A = activation bytes): forward stats + apply 3A (4A + A/16 with a residual: the ReLU bit
mask); backward with the ReLU mask recomputed from x 5A (reduce: dy, x; dx: dy, x -> dx); backward with a residual
6A + A/8 (reduce: dy, x, bits; dx: dy, x, bits -> dx, dres).  One JSON object per shape on stdout plus a summary line.

    python benchmarks/bn_bench.py [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

# (H*W, C, calls per step): every BN layer of torchvision-layout ResNet-50 (stem, 3/4/6/3 bottlenecks + downsample)
RESNET50_BN = [
    (112 * 112, 64, 1),
    (56 * 56, 64, 6), (56 * 56, 256, 4), (56 * 56, 128, 1),
    (28 * 28, 128, 7), (28 * 28, 512, 5), (28 * 28, 256, 1),
    (14 * 14, 256, 11), (14 * 14, 1024, 7), (14 * 14, 512, 1),
    (7 * 7, 512, 5), (7 * 7, 2048, 4),
]


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    _lib.require()
    o = _lib.ops()
    rows, tot = [], {"copy": 0.0, "fwd": 0.0, "fwd_res": 0.0, "bwd_xmask": 0.0, "bwd_res": 0.0}
    for hw, c, calls in RESNET50_BN:
        m = args.batch * hw
        x = torch.randn(m, c, device="cuda", dtype=torch.bfloat16)
        r = torch.randn_like(x)
        dy = torch.randn_like(x)
        w = torch.rand(c, device="cuda", dtype=torch.bfloat16) + 0.5
        b = torch.randn(c, device="cuda", dtype=torch.bfloat16) * 0.1
        rm = torch.zeros(c, device="cuda")
        rv = torch.ones(c, device="cuda")
        bits = torch.empty(m * c // 8, device="cuda", dtype=torch.uint8)   # ReLU-after-residual mask (1 bit/elem)
        a = x.numel() * 2
        t = {
            "copy": timeit(lambda: x.clone()),
            "fwd": timeit(lambda: o.bn_act_fwd(x, None, w, b, rm, rv, 0.1, 1e-5, True, None, None)),
            "fwd_res": timeit(lambda: o.bn_act_fwd(x, r, w, b, rm, rv, 0.1, 1e-5, True, None, None, bits)),
        }
        y, mean, invstd, ss = o.bn_act_fwd(x, None, w, b, rm, rv, 0.1, 1e-5, True, None, None)
        t["bwd_xmask"] = timeit(lambda: o.bn_act_bwd(dy, x, x, mean, invstd, w, True, False, True, ss, None, None))
        t["bwd_res"] = timeit(lambda: o.bn_act_bwd(dy, y, x, mean, invstd, w, True, True, True, None, None, None,
                                                   bits))
        traffic = {"copy": 2, "fwd": 3, "fwd_res": 4 + 1 / 16, "bwd_xmask": 5, "bwd_res": 6 + 1 / 8}
        row = {"M": m, "C": c, "calls": calls, "MB": round(a / 1e6, 1)}
        for k, ms in t.items():
            row[k + "_us"] = round(ms * 1e3, 1)
            row[k + "_GBs"] = round(traffic[k] * a / ms / 1e6, 0)
            tot[k] += ms * calls
        rows.append(row)
        print(json.dumps(row), flush=True)
        del x, r, dy, y
    # the stem's max pooling (ops/pool.py) vs ATen, forward + backward
    from distributed_pytorch_hpc_amd.ops.pool import max_pool3s2

    xs = torch.randn(args.batch, 64, 112, 112, device="cuda", dtype=torch.bfloat16)
    xs = xs.contiguous(memory_format=torch.channels_last).requires_grad_()
    gy = torch.randn(args.batch, 64, 56, 56, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    pool = {}
    for name, fn in (("dph", max_pool3s2), ("aten", lambda t: torch.nn.functional.max_pool2d(t, 3, 2, 1))):
        pool[name + "_fwd_us"] = round(timeit(lambda: fn(xs.detach())) * 1e3, 1)
        pool[name + "_fwd_bwd_us"] = round(timeit(lambda: fn(xs).backward(gy)) * 1e3, 1)
    print(json.dumps({"stem_maxpool": pool}), flush=True)
    summ = {k + "_ms_per_step_if_all_layers": round(v, 3) for k, v in tot.items()}
    summ["stem_maxpool"] = pool
    print(json.dumps(summ), flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump({"rows": rows, "summary": summ}, fh, indent=1)


if __name__ == "__main__":
    main()
