#!/usr/bin/env python3
"""Clock- and power-normalised A/B of the projection GEMMs: hipBLASLt vs the CDNA4 NT kernel on Llama-2-7B shapes, each arm run back to back for --seconds so the chip settles at the clock its power
limit allows, with the GPU's clock, socket power and energy sampled over exactly that window
(distributed_pytorch_hpc_amd/utils/telemetry.py).  Reports TFLOP/s, median SCLK, median power, TFLOP per joule and
the fraction of the window the package power limit (PPT) was active.  Interleaved rounds, one process
(cdna_hip_programming.md rule 24); random operands (rule 25).

    python benchmarks/probes/gemm_power.py [--shapes w13,w2,wqkv,w13.dgrad] [--seconds 2] [--rounds 2]
    python benchmarks/probes/gemm_power.py --shapes w13.wgrad,w2.wgrad --arms tn,blaslt,blaslt_kc

A ``.wgrad`` shape is the weight gradient dW[N, K] = dY^T X over the tokens (dY [T, N], X [T, K]): ``tn`` = the
framework's CDNA4 kernel (csrc/gemm.hip, bf16 out), ``blaslt`` = hipBLASLt on the same token-major operands,
``blaslt_kc`` = hipBLASLt on pre-transposed K-contiguous copies (the transposes not counted).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402
from distributed_pytorch_hpc_amd.utils.telemetry import GpuTelemetry  # noqa: E402

SHAPES = {"wqkv": (12288, 4096), "wo": (4096, 4096), "w13": (22016, 4096), "w2": (4096, 11008),
          "output": (32000, 4096), "w13.dgrad": (4096, 22016), "w2.dgrad": (11008, 4096)}
for _n in ("wqkv", "wo", "w13", "w2", "output"):
    SHAPES[_n + ".wgrad"] = SHAPES[_n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--shapes", default="w13,w2,wqkv,w13.dgrad")
    ap.add_argument("--arms", default="blaslt,nt16")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    _lib.require()
    ops = torch.ops.dph
    tel = GpuTelemetry(0, period=0.05)
    out = []
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        wg = name.endswith(".wgrad")
        x = torch.randn(a.tokens, K, device="cuda").to(torch.bfloat16)
        w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
        if wg:
            dy = torch.randn(a.tokens, N, device="cuda").to(torch.bfloat16)
            c = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
            dyT, xT = dy.t().contiguous(), x.t().contiguous()
        flop = 2.0 * a.tokens * N * K
        for rnd in range(a.rounds):
            for arm in a.arms.split(","):
                if wg and arm == "tn":
                    fn = lambda: ops.gemm_tn_(c, dy, x, False)  # noqa: E731
                elif wg and arm == "blaslt":
                    fn = lambda: torch.matmul(dy.t(), x)  # noqa: E731
                elif wg and arm == "blaslt_kc":
                    fn = lambda: torch.matmul(dyT, xT.t())  # noqa: E731
                elif arm == "blaslt":
                    fn = lambda: torch.matmul(x, w.t())  # noqa: E731
                elif arm in ("nt4", "nt4n", "nt4p", "nt4h"):   # 4-wave / 256-AGPR gemm_nt4_k, PIPE 1 / 0 / 2 / 3
                    v = {"nt4": 5, "nt4n": 4, "nt4p": 6, "nt4h": 7}[arm]

                    def fn(v=v):
                        old = ops.gemm_nt_variant(v)
                        y = ops.gemm_nt(x, w)
                        ops.gemm_nt_variant(old)
                        return y
                    if rnd == 0:   # numerics against hipBLASLt on the same operands
                        ref = torch.matmul(x, w.t()).float()
                        err = ((fn().float() - ref).norm() / ref.norm()).item()
                        print(json.dumps({"shape": name, "arm": arm, "rel_err_vs_blaslt": err}), flush=True)
                        if not err < 1e-2:
                            raise SystemExit(f"{arm} wrong on {name}: rel err {err}")
                else:   # the CDNA4 NT kernel (16x16x32; the 32x32x16 form measured in round 5 was removed)
                    fn = lambda: ops.gemm_nt(x, w)  # noqa: E731
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                # size the window from one timed call
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                n = max(5, int(a.seconds / max(time.perf_counter() - t0, 1e-4)))
                tel.mark("s")
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(n):
                    fn()
                e.record()
                e.synchronize()
                tel.mark("e")
                ms = s.elapsed_time(e) / n
                summ = tel.summary("s", "e", flops=flop * n)
                row = {"shape": name, "arm": arm, "round": rnd, "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1),
                       "sclk_mhz": (summ.get("sclk_mhz") or {}).get("median"),
                       "power_w": (summ.get("power_w") or {}).get("median"),
                       "tflop_per_joule": summ.get("tflop_per_joule"), "ppt_frac": summ.get("ppt_limited_frac")}
                out.append(row)
                print(json.dumps(row), flush=True)
        del x, w
        if wg:
            del dy, c, dyT, xT
    tel.stop()
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
