"""The ring-attention merge fused into the flash forward epilogue (flash_attn_fwd_merge_): a ring of P K/V blocks
simulated on one GPU -- the contiguous and the zig-zag causal schedules of parallel/context_parallel.py -- against an
fp32 full-sequence reference, and against the eager (flash + logaddexp merge) path it replaces (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, causal=True):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, device=DEV, dtype=torch.bool).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    return (torch.softmax(s, -1) @ vf).transpose(1, 2), lse


@pytest.mark.parametrize("P,D", [(4, 128), (3, 64), (8, 128)])
def test_fused_ring_merge_contiguous(dph_native, P, D):
    B, H, C = 2, 4, 128                       # C tokens per rank
    g = torch.Generator(device=DEV).manual_seed(0)
    q, k, v = (torch.randn(B, P * C, H, D, device=DEV, generator=g).to(torch.bfloat16) for _ in range(3))
    ro, rl = _ref(q, k, v)
    scale = 1 / math.sqrt(D)
    for r in range(P):                       # rank r: queries of chunk r, K/V chunks r, r-1, ..., 0 (ring order)
        qs = q[:, r * C:(r + 1) * C]
        acc = torch.zeros(B, C, H, D, device=DEV)
        lse = torch.full((B, H, C), float("-inf"), device=DEV)
        for i in range(P):
            j = (r - i) % P
            if j > r:
                continue
            ks, vs = k[:, j * C:(j + 1) * C], v[:, j * C:(j + 1) * C]
            dph_native.flash_attn_fwd_merge_(qs, ks, vs, scale, j == r, acc, lse)
        assert (acc - ro[:, r * C:(r + 1) * C]).abs().max() < 2e-2
        assert (lse - rl[:, :, r * C:(r + 1) * C]).abs().max() < 1e-3


def test_fused_ring_merge_views_and_eager_parity(dph_native):
    """Row-slice views of the accumulators (the zig-zag schedule merges into the second half only) and the same
    numbers as the eager merge of parallel/context_parallel.py (flash o rounded to bf16, then logaddexp)."""
    from distributed_pytorch_hpc_amd.parallel.context_parallel import _merge

    B, H, S, D = 1, 8, 256, 128
    g = torch.Generator(device=DEV).manual_seed(1)
    q, k1, v1, k2, v2 = (torch.randn(B, S, H, D, device=DEV, generator=g).to(torch.bfloat16) for _ in range(5))
    scale = 1 / math.sqrt(D)
    c = S // 2
    acc = torch.zeros(B, S, H, D, device=DEV)
    lse = torch.full((B, H, S), float("-inf"), device=DEV)
    dph_native.flash_attn_fwd_merge_(q, k1, v1, scale, True, acc, lse)                   # diagonal block
    dph_native.flash_attn_fwd_merge_(q[:, c:], k2, v2, scale, False, acc[:, c:], lse[:, :, c:])   # later chunk
    o_e = torch.zeros(B, S, H, D, device=DEV)
    l_e = torch.full((B, H, S), float("-inf"), device=DEV)
    ob, lb = dph_native.flash_attn_fwd(q, k1, v1, scale, True)
    o_e, l_e = _merge(o_e, l_e, ob, lb)
    ob, lb = dph_native.flash_attn_fwd(q[:, c:], k2, v2, scale, False)
    o2, l2 = _merge(o_e[:, c:], l_e[:, :, c:], ob, lb)
    o_e[:, c:], l_e[:, :, c:] = o2, l2
    assert (acc - o_e).abs().max() < 1e-2            # eager rounds each block's o to bf16 first
    assert (lse - l_e).abs().max() < 1e-4
