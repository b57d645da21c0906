#!/usr/bin/env python3
"""One ring-attention step on one GPU: flash forward + eager online-softmax merge (logaddexp, exp, two scaled adds
over the fp32 accumulator) vs the merge fused into the flash epilogue (flash_attn_fwd_merge_).  Shape of a
context-parallel shard: --cp 8 of a --seq 32768 sequence, 32 heads x 128.

    python benchmarks/ring_merge_bench.py [--seq 32768] [--cp 8] [--json out.json]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.context_parallel import _merge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=32768)
    ap.add_argument("--cp", type=int, default=8)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    _lib.require()
    ops = torch.ops.dph
    C, H, D = a.seq // a.cp, a.heads, 128
    q, k, v = (torch.randn(1, C, H, D, device="cuda").to(torch.bfloat16) for _ in range(3))
    acc = torch.zeros(1, C, H, D, device="cuda")
    lse = torch.full((1, H, C), float("-inf"), device="cuda")
    scale = 1 / math.sqrt(D)

    def eager():
        ob, lb = ops.flash_attn_fwd(q, k, v, scale, False)
        o2, l2 = _merge(acc, lse, ob, lb)
        acc.copy_(o2)
        lse.copy_(l2)

    def fused():
        ops.flash_attn_fwd_merge_(q, k, v, scale, False, acc, lse)

    def flash_only():
        ops.flash_attn_fwd(q, k, v, scale, False)

    res = {}
    for name, fn in (("flash_only", flash_only), ("eager_merge", eager), ("fused_merge", fused)) * 2:
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        res[name] = min(res.get(name, 1e9), s.elapsed_time(e) / a.iters)
    print(json.dumps({"shape": {"local_seq": C, "heads": H, "head_dim": D}, "ms_per_step": res}))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
