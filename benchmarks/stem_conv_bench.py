#!/usr/bin/env python3
"""ResNet stem convolution (7x7 / 2 / 3, 64 filters, B x 224 x 224, channels-last bf16) through MIOpen with the
input's 3 channels as is or zero-padded to 4 / 8 (weight gradient only, as in training: the image needs no
gradient).  Find mode on, like the drivers.  Prints ms for forward and forward + weight gradient per channel count,
then the same for the framework's chunk-tap stem (ops/conv.py StemConv2d on csrc/conv3x3.hip conv3_k GEN = 2)."""
import os
import json
import sys

import torch
import torch.nn.functional as F


def timeit(fn, iters=20):
    for _ in range(3):
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
    torch.backends.cudnn.benchmark = True
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    res = {}
    for c in (3, 4, 8):
        x = torch.randn(B, c, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(64, c, 7, 7, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_()
        gy = torch.randn(B, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        fwd = timeit(lambda: F.conv2d(x, w.detach(), None, 2, 3))
        both = timeit(lambda: F.conv2d(x, w, None, 2, 3).backward(gy))
        res[c] = {"fwd_ms": round(fwd, 3), "fwd_wgrad_ms": round(both, 3)}
        print(json.dumps({"channels": c, **res[c]}), flush=True)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.ops.conv import StemConv2d

    _lib.require()
    conv = StemConv2d(3, 64, 7, 2, 3, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(B, 3, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(B, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        fwd = timeit(lambda: conv(x))
    both = timeit(lambda: conv(x).backward(gy))
    res["dph"] = {"fwd_ms": round(fwd, 3), "fwd_wgrad_ms": round(both, 3)}
    print(json.dumps({"dph_chunk_tap_stem": res["dph"]}), flush=True)


if __name__ == "__main__":
    main()
