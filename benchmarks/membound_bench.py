#!/usr/bin/env python3
"""HBM bandwidth of the memory-bound kernels at the Llama-2-7B bench sizes (T = 32768 tokens, tensors larger
than the 256 MB Infinity Cache), in GB/s of compulsory traffic (fraction of the measured 6.3 TB/s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


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
    _lib.require()
    o = _lib.ops()
    T, D, F = 32768, 4096, 11008
    res = {}
    big = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)   # 1.44 GB: far beyond the Infinity Cache
    res["copy_clone"] = 2 * big.numel() * 2 / timeit(lambda: big.clone()) / 1e6
    dst = torch.empty_like(big)
    res["copy_"] = 2 * big.numel() * 2 / timeit(lambda: dst.copy_(big)) / 1e6
    del big, dst
    x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.ones(D, device="cuda", dtype=torch.bfloat16)
    n = x.numel() * 2
    res["rmsnorm_add_fwd"] = 4 * n / timeit(lambda: o.rmsnorm_fwd(x, w, 1e-5, r)) / 1e6
    y, rstd, h = o.rmsnorm_fwd(x, w, 1e-5, r)
    res["rmsnorm_bwd"] = 3 * n / timeit(lambda: o.rmsnorm_bwd(y, x, w, rstd, None)) / 1e6
    res["rmsnorm_bwd_dres"] = 4 * n / timeit(lambda: o.rmsnorm_bwd(y, x, w, rstd, r)) / 1e6
    del y, h
    g = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    m = T * F * 2
    res["swiglu_fwd"] = 3 * m / timeit(lambda: o.swiglu_fwd(g)) / 1e6
    res["swiglu_bwd"] = 5 * m / timeit(lambda: o.swiglu_bwd(dy, g)) / 1e6
    del g, dy
    qkv = torch.randn(T, 3 * D, device="cuda", dtype=torch.bfloat16)
    from distributed_pytorch_hpc_amd.ops.rope import precompute_rope_tables
    cos, sin = precompute_rope_tables(128, 8192, 1e4, "cuda")
    try:
        q = qkv.view(8, 4096, 3 * D)[:, :, :2 * D]
        res["rope_qk_inplace"] = 2 * (T * 2 * D * 2) / timeit(lambda: o.rope_(q.view(8, 4096, 64, 128), cos, sin, 0, False)) / 1e6
    except Exception as e:  # signature differences are reported, not fatal
        res["rope_error"] = str(e)[:200]
    nparam = 1 << 28
    p = torch.randn(nparam, device="cuda")
    mm, vv = torch.zeros_like(p), torch.zeros_like(p)
    gg = torch.randn(nparam, device="cuda", dtype=torch.bfloat16)
    pb = torch.empty(nparam, device="cuda", dtype=torch.bfloat16)
    res["adamw"] = nparam * 28 / timeit(lambda: o.adamw_step_(p, mm, vv, gg, pb, 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.5, None)) / 1e6
    out = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}
    out.update({k + "_frac": round(v / 6300, 3) for k, v in res.items() if isinstance(v, float)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
