"""Flash-attention forward + backward numerics against the fp32 reference for a few shapes, in a fresh process.

The kernels' launch configuration is read from the environment once per process (DPH_ATTN_WAVES: 4- or 8-wave
workgroups), so tests/test_kernels_gpu.py runs this script as a child process to cover the non-default variant.
Prints one JSON line with the worst relative errors; exits 1 if any exceeds the tolerances of test_flash_attention.
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd import ops  # noqa: E402
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402
from distributed_pytorch_hpc_amd.ops import attention as attn_mod  # noqa: E402

CASES = [  # B, Sq, Sk, Hq, Hkv, D, causal -- d >= 64 (the 8-wave variants), ragged lengths, GQA
    (2, 256, 256, 4, 4, 128, True),
    (1, 300, 300, 4, 4, 128, False),
    (2, 200, 200, 8, 2, 64, True),
    (1, 64, 192, 2, 2, 64, True),
    (1, 520, 520, 2, 1, 128, True),
    (2, 1000, 1000, 4, 2, 128, True),
    (1, 192, 64, 2, 2, 128, True),
    (1, 300, 77, 2, 2, 64, False),
    (1, 77, 300, 2, 1, 128, True),
    (1, 2048, 2048, 2, 2, 128, True),   # with spiked keys: forces the lazy-rescale branch mid-sequence
]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    _lib.require()
    worst = {"o": 0.0, "dq": 0.0, "dk": 0.0, "dv": 0.0}
    for B, Sq, Sk, Hq, Hkv, D, causal in CASES:
        torch.manual_seed(9)
        q = torch.randn(B, Sq, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        if Sq == 2048:
            with torch.no_grad():
                dirn = q.float().mean(1)
                dirn = dirn / dirn.norm(dim=-1, keepdim=True)
                k[:, 700] = (dirn * 30).to(torch.bfloat16)
                k[:, 1500] = (dirn * 60).to(torch.bfloat16)
        o = ops.flash_attention(q, k, v, causal=causal)
        qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
        orf = attn_mod.attention_reference(qr, kr, vr, causal, 1.0 / math.sqrt(D))
        do = torch.randn_like(o)
        o.backward(do)
        orf.backward(do.float())
        for key, a, b in (("o", o, orf), ("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
            worst[key] = max(worst[key], rel(a, b))
    torch.cuda.synchronize()
    ok = worst["o"] < 2e-2 and max(worst["dq"], worst["dk"], worst["dv"]) < 3e-2
    print(json.dumps({"waves": os.environ.get("DPH_ATTN_WAVES", "default"), "worst_rel_err": worst, "ok": ok}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
