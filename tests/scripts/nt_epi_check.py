"""Child process for test_gemm_nt_gpu.py::test_gemm_nt_epilogue_forms_bitwise: runs the forward GEMM (STORE) and the
w13 projection with SwiGLU (SWIGLU), the w2 input gradient with the SwiGLU backward (DSWIGLU) on fixed inputs and prints a hash of the output bytes; the
parent runs it under DPH_NT_EPI=reg (register epilogue) and the default (LDS epilogue) and compares."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_hpc_amd.ops import _lib  # noqa: E402

_lib.require()
ops = torch.ops.dph
h = hashlib.sha256()
for M, N, K in [(512, 768, 320), (256, 1024, 4096)]:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    x13 = (2 * torch.randn(M, 2 * N, device="cuda", generator=g)).to(torch.bfloat16)
    h.update(ops.gemm_nt(a, b).cpu().view(torch.int16).numpy().tobytes())
    h.update(ops.gemm_nt_dswiglu(a, b, x13).cpu().view(torch.int16).numpy().tobytes())
    for t in ops.gemm_nt_swiglu(a, b):   # b as [W1; W3] of N / 2 hidden units
        h.update(t.cpu().view(torch.int16).numpy().tobytes())
    # the wqkv projection with RoPE on q / k (head dim 64 or 128, 2 of 3 thirds rotated)
    from distributed_pytorch_hpc_amd.models.llama2 import rope_tables
    hd = 64 if N == 768 else 128
    cos, sin = rope_tables(hd, 2 * M, 10000.0, torch.device("cuda"))
    n_rot = (2 * N // 3) // hd * hd
    h.update(ops.gemm_nt_rope(a, b, cos, sin, M // 2, hd, n_rot, 3).cpu().view(torch.int16).numpy().tobytes())
print(h.hexdigest())
