#!/usr/bin/env python3
"""FP8 probe 2: e5m2 x e4m3 (gradient x weight) support, the weight-gradient shape (K = tokens) with transposed
operands, out= into a preallocated bf16 buffer, and the cost of torch-side quantisation of a [T, 4096] activation."""
import json

import torch


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
    res = {}
    one = torch.ones((), device="cuda", dtype=torch.float32)
    T = 32768
    # dgrad: dX [T, 4096] = dY [T, 12288] . W [12288, 4096]  ->  A = dY (e5m2), B^T = W^T [4096, 12288] (e4m3)
    dy = torch.randn(T, 12288, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(4096, 12288, device="cuda", dtype=torch.bfloat16)
    for fa, fb in (("float8_e5m2", "float8_e4m3fn"), ("float8_e4m3fn", "float8_e5m2"), ("float8_e5m2", "float8_e5m2")):
        try:
            a8, b8 = dy.to(getattr(torch, fa)), wt.to(getattr(torch, fb))
            out = torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            ref = a8.float() @ b8.float().t()
            res[f"{fa}x{fb}"] = {"relerr": ((out.float() - ref).norm() / ref.norm()).item(),
                                 "tflops": 2.0 * T * 12288 * 4096 / timeit(lambda: torch._scaled_mm(
                                     a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)) / 1e9}
        except Exception as ex:
            res[f"{fa}x{fb}"] = f"{type(ex).__name__}: {str(ex)[:150]}"
    del dy, wt
    # wgrad: dW [12288, 4096] = dY^T X with K = T: A = dY^T [12288, T], B^T = X^T [4096, T]
    dyt = torch.randn(12288, T, device="cuda", dtype=torch.bfloat16).to(torch.float8_e4m3fn)
    xt = torch.randn(4096, T, device="cuda", dtype=torch.bfloat16).to(torch.float8_e4m3fn)
    outbuf = torch.empty(12288, 4096, device="cuda", dtype=torch.bfloat16)
    try:
        ms = timeit(lambda: torch._scaled_mm(dyt, xt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                             out=outbuf))
        res["wgrad_e4m3_out"] = {"tflops": 2.0 * T * 12288 * 4096 / ms / 1e9}
    except Exception as ex:
        res["wgrad_e4m3_out"] = f"{type(ex).__name__}: {str(ex)[:150]}"
    del dyt, xt
    # torch-side quantisation of a [T, 4096] bf16 activation (amax + scale + cast, and a transposed copy)
    x = torch.randn(T, 4096, device="cuda", dtype=torch.bfloat16)

    def q():
        s = 448.0 / x.abs().amax().float().clamp(min=1e-12)
        return (x.float() * s).to(torch.float8_e4m3fn)

    res["torch_quant_ms"] = timeit(q)
    res["torch_quant_transpose_ms"] = timeit(lambda: q().t().contiguous())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
