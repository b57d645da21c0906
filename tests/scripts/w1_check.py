"""1x1 weight-gradient GEMM (ts_gemm_tn_: dW = dY^T X over channels-last pixels) against an fp32 reference, in a
child process of tests/test_kernels_gpu.py (a kernel fault ends the child, not the test session).  Shapes cover both output tile widths,
64- and 128-wide k' tiles, a pixel count that leaves a ragged last chunk / step, and accumulation into bf16 and fp32.
Prints one JSON line; exits 1 on a tolerance miss."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

CASES = [  # M pixels, Cout (N), Cin (K), out dtype, accumulate
    (2 * 56 * 56, 64, 64, torch.float32, False),
    (3 * 28 * 28 + 17, 128, 512, torch.float32, True),
    (8 * 14 * 14, 512, 1024, torch.bfloat16, False),
    (5 * 7 * 7 + 3, 2048, 512, torch.float32, False),
    (4 * 28 * 28, 512, 128, torch.bfloat16, True),
    (16 * 56 * 56, 256, 64, torch.float32, False),
]


def main():
    _lib.require()
    ops = _lib.ops()
    g = torch.Generator(device="cuda").manual_seed(7)
    worst = 0.0
    for M, N, K, dt, acc in CASES:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
        base = torch.randn(N, K, device="cuda", generator=g).to(dt)
        out = base.clone()
        ops.ts_gemm_tn_(out, dy, x, acc)
        ref = dy.float().t() @ x.float() + (base.float() if acc else 0.0)
        err = ((out.float() - ref).norm() / ref.norm()).item()
        worst = max(worst, err / (1e-2 if dt == torch.bfloat16 else 1e-4))
        print(json.dumps({"M": M, "N": N, "K": K, "dtype": str(dt), "acc": acc, "rel_err": err}), flush=True)
    ok = worst <= 1.0
    print(json.dumps({"ok": ok, "worst_over_tol": worst}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
