#!/usr/bin/env python3
"""How far bf16 whole-network gradients land from fp32 (ResNet-50 under the world-1 FSDP engine, SimpleUNet under
DDP), for the framework's kernels and for stock ATen / MIOpen bf16, per parameter: the conditioning data behind the
tolerances of tests/test_whole_net_grad_gpu.py.  Random-init BatchNorm-ReLU networks amplify rounding, so the probe
sweeps the residual-branch gain (each bottleneck's bn3 gamma) and every BatchNorm's shift (beta: how many ReLU inputs
are clipped) to find a regime where bf16 error is small.

    python benchmarks/probes/wholenet_conditioning.py [--gammas 1 0.25 0.05] [--betas 1 3] [--unet]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gammas", type=float, nargs="*", default=[1.0, 0.25, 0.05])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=112)
    ap.add_argument("--unet", action="store_true")
    ap.add_argument("--betas", type=float, nargs="*", default=[None], help="BatchNorm shift (none = 0 init)")
    ap.add_argument("--rows", action="store_true", help="also print every parameter's row")
    a = ap.parse_args()
    import test_whole_net_grad_gpu as t

    for beta in a.betas:
        for gamma in a.gammas:
            rows = t.resnet_rows(gamma, a.batch, a.res, beta)
            print(json.dumps({"model": "resnet50", "gamma": gamma, "beta": beta, **t.summarize(rows)}), flush=True)
            if a.rows:
                for r in rows["rows"]:
                    print("  %-32s rel %.4f cos %.5f | aten bf16 rel %.4f cos %.5f | |g32| %.3e" % r[:6])
        if a.unet:
            rows = t.unet_rows(beta=beta)
            print(json.dumps({"model": "simple_unet", "beta": beta, **t.summarize(rows)}), flush=True)


if __name__ == "__main__":
    main()
