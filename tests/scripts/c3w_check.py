"""3x3 / strided / stem weight gradients on the LDS-DMA c3w_k kernel against an fp32 reference, in a child process
of tests/test_kernels_gpu.py.  Covers the stride-1 3x3 implicit GEMM (ts_gemm_tn_ with H, W), the gathered strided 3x3 / 1x1
(StridedConv2d) and the chunk-tap RGB stem, with ragged pixel counts.
Prints one JSON line; exits 1 on a tolerance miss."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402
from distributed_pytorch_hpc_amd.ops.conv import StemConv2d, StridedConv2d  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    _lib.require()
    torch.manual_seed(11)
    res = {}
    # stride-1 3x3: dW[co, tap * cin + c] over channels-last pixels
    for B, H, W, C, Co in [(2, 14, 14, 64, 64), (3, 9, 11, 128, 256), (8, 28, 28, 128, 128)]:
        x = torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(B, H, W, Co, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(Co, 9 * C, device="cuda")
        _lib.ops().ts_gemm_tn_(out, dy.view(-1, Co), x.view(-1, C), False, H, W)
        ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (Co, C, 3, 3), dy.permute(0, 3, 1, 2).float(),
                                          padding=1)
        res[f"s1_{B}x{H}x{W}x{C}->{Co}"] = rel(out.view(Co, 3, 3, C).permute(0, 3, 1, 2), ref)
    # strided 3x3 / 1x1 (gathered geometry)
    for k, B, C, Co, H, W in [(3, 2, 64, 64, 16, 16), (3, 3, 128, 128, 15, 15), (1, 2, 256, 512, 14, 14),
                              (1, 1, 512, 1024, 28, 28)]:
        conv = StridedConv2d(C, Co, k, 2, k // 2, bias=False).cuda().to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        x = torch.randn(B, C, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = conv(x)
        g = torch.randn_like(y.float())
        y.float().backward(g)
        wr = conv.weight.detach().float().requires_grad_()
        F.conv2d(x.float(), wr, stride=2, padding=k // 2).backward(g)
        res[f"strided{k}_{B}x{C}->{Co}@{H}x{W}"] = rel(conv.weight.grad, wr.grad)
    # chunk-tap stem
    for B, H, W in [(2, 64, 64), (3, 37, 50)]:
        conv = StemConv2d(3, 64, 7, 2, 3, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        x = torch.randn(B, 3, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = conv(x)
        g = torch.randn_like(y.float())
        y.float().backward(g)
        wr = conv.weight.detach().float().requires_grad_()
        F.conv2d(x.float(), wr, stride=2, padding=3).backward(g)
        res[f"stem_{B}x{H}x{W}"] = rel(conv.weight.grad, wr.grad)
    worst = max(res.values())
    ok = worst < 1e-2
    print(json.dumps({"ok": ok, "worst": worst, **res}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
