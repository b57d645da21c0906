#!/usr/bin/env python3
"""Run the flash-attention kernels on one Llama-2-7B shape a few times (for rocprofv3 counter collection)
and print their TFLOP/s."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd import ops  # noqa: E402
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=8)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--which", default="fwd,bwd")
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--packed", action="store_true",
                    help="q / k / v as views of one [B, S, 3 H D] projection output (the Llama step's layout)")
    ap.add_argument("--variant", type=int, default=0, help="attention kernel forms for D 128: 0 = 32x32x16 (default), "
                                                            "2 = 16x16x32")
    ap.add_argument("--sustain", type=float, default=0.0,
                    help="also loop each kernel for this many seconds under the GPU telemetry sampler (clock, power, "
                         "package-power residency, TFLOP/J)")
    a = ap.parse_args()
    _lib.require()
    _lib.ops().attn_variant(a.variant)
    causal = not a.noncausal
    if a.packed:
        qkv = torch.randn(a.b, a.s, 3 * a.h * a.d, device="cuda", dtype=torch.bfloat16)
        q, k, v = (qkv[:, :, i * a.h * a.d:(i + 1) * a.h * a.d].view(a.b, a.s, a.h, a.d) for i in range(3))
    else:
        q, k, v = (torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    do = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(a.d)
    o, lse = ops.flash_fwd(q, k, v, scale, causal)
    flops = 4 * a.b * a.h * a.s * a.s * a.d * (0.5 if causal else 1.0)
    for which in a.which.split(","):
        fn = (lambda: ops.flash_fwd(q, k, v, scale, causal)) if which == "fwd" else \
            (lambda: _lib.ops().flash_attn_bwd(do, q, k, v, o, lse, scale, causal))
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        f = flops * (2.5 if which == "bwd" else 1.0)
        print(f"{which}: {ms:.3f} ms  {f / ms / 1e9:.1f} TFLOP/s", flush=True)
        if a.sustain > 0:
            from distributed_pytorch_hpc_amd.utils.telemetry import GpuTelemetry

            n = max(1, int(a.sustain * 1e3 / ms))
            tel = GpuTelemetry(torch.cuda.current_device(), period=0.05)
            tel.mark("start")
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            tel.mark("end")
            tel.stop()
            summ = tel.summary("start", "end", flops=f * n)
            keep = ("sclk_mhz", "power_w", "avg_power_w", "tflop_per_joule", "ppt_limited_frac")
            print(f"{which} sustained x{n}: " + json.dumps({k: summ.get(k) for k in keep}), flush=True)


if __name__ == "__main__":
    main()
