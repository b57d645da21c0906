#!/usr/bin/env python3
"""Probe: does torch._scaled_mm run OCP fp8 (e4m3fn / e5m2) GEMMs on this gfx950 build, and how fast on the
Llama-2-7B projection shapes vs bf16 torch.mm (forward NT layout)?  Prints one JSON line."""
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
    res = {"torch": torch.__version__, "hip": torch.version.hip, "arch": torch.cuda.get_device_properties(0).gcnArchName}
    T = 32768
    for name, (N, K) in {"wqkv": (12288, 4096), "w13": (22016, 4096), "w2": (4096, 11008)}.items():
        a = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * T * N * K
        row = {"bf16_tflops": flop / timeit(lambda: a @ w.t()) / 1e9}
        for fmt in ("float8_e4m3fn", "float8_e4m3fnuz"):
            dt = getattr(torch, fmt, None)
            if dt is None:
                continue
            try:
                a8, w8 = a.to(dt), w.to(dt)
                one = torch.ones((), device="cuda", dtype=torch.float32)
                out = torch._scaled_mm(a8, w8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                ref = (a8.float() @ w8.float().t())
                row[fmt + "_relerr"] = ((out.float() - ref).norm() / ref.norm()).item()
                row[fmt + "_tflops"] = flop / timeit(lambda: torch._scaled_mm(a8, w8.t(), scale_a=one, scale_b=one,
                                                                               out_dtype=torch.bfloat16)) / 1e9
            except Exception as ex:  # report, do not fail
                row[fmt + "_error"] = f"{type(ex).__name__}: {str(ex)[:160]}"
        res[name] = row
        del a, w
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
