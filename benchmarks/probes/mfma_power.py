#!/usr/bin/env python3
"""Energy per FLOP of the two bf16 MFMA shapes with no memory traffic: runs the compiled mfma_power.hip binary for
each shape (a child process) while this process samples the GPU (utils/telemetry.py), interleaved over rounds, and
prints one JSON line per run with TFLOP/s, clock, power and TFLOP/J.

    hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_power benchmarks/probes/mfma_power.hip
    python benchmarks/probes/mfma_power.py --bin /tmp/mfma_power [--seconds 3] [--rounds 2]
"""
import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.utils.telemetry import GpuTelemetry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bin", required=True)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    for rnd in range(a.rounds):
        for shape in (32, 16):
            tel = GpuTelemetry(0, period=0.05)
            tel.mark("start")
            out = subprocess.run([a.bin, str(shape), str(a.seconds)], capture_output=True, text=True, timeout=120)
            tel.mark("end")
            tel.stop()
            res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
            s = tel.summary("start", "end")
            e = s.get("energy_j")
            res.update({"round": rnd, "sclk_mhz": (s.get("sclk_mhz") or {}).get("median"),
                        "power_w": s.get("avg_power_w"), "ppt_frac": s.get("ppt_limited_frac")})
            if res["power_w"]:
                res["tflop_per_joule"] = round(res["tflops"] / res["power_w"], 4)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
