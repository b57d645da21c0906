"""Attention dropout in the CDNA4 flash kernels (csrc/attention.hip / attention_bwd.hip DROP instantiations).

The keep mask is a counter hash the kernels regenerate; ``ops.attention.dropout_mask`` rebuilds it on the host, so
the kernels are checked against an fp32 PyTorch reference of dropout attention with exactly that mask.
"""
import math

import pytest
import torch

from distributed_pytorch_hpc_amd.ops.attention import dropout_mask


def test_dropout_mask_rate_and_independence():
    m = dropout_mask(2, 4, 256, 256, 0.1, seed=1234)
    keep = m.float().mean().item()
    assert abs(keep - 0.9) < 0.005
    # different heads / seeds give (nearly) uncorrelated masks
    assert (m[0, 0] ^ m[0, 1]).float().mean().item() > 0.15
    m2 = dropout_mask(2, 4, 256, 256, 0.1, seed=1235)
    assert (m ^ m2).float().mean().item() > 0.15
    assert dropout_mask(1, 1, 8, 8, 0.0, seed=3).all()


def _reference(q, k, v, mask, p, causal, scale):
    """fp32 dropout attention on [B, S, H, D] with keep mask [B, Hq, Sq, Sk]."""
    hq, hk = q.shape[2], k.shape[2]
    if hq != hk:
        k = k.repeat_interleave(hq // hk, dim=2)
        v = v.repeat_interleave(hq // hk, dim=2)
    qt, kt, vt = (t.float().transpose(1, 2) for t in (q, k, v))
    s = qt @ kt.transpose(-1, -2) * scale
    if causal:
        sq, sk = s.shape[-2:]
        i = torch.arange(sq, device=s.device)[:, None]
        j = torch.arange(sk, device=s.device)[None, :]
        s = s.masked_fill(j > i + (sk - sq), float("-inf"))
    pr = torch.softmax(s, -1) * mask / (1 - p)
    return (pr @ vt).transpose(1, 2)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal,p", [
    (2, 128, 8, 8, 32, False, 0.1),     # pipeline transformer's attention (dim 256, 8 heads)
    (1, 256, 4, 4, 64, True, 0.2),
    (2, 200, 4, 2, 128, True, 0.1),     # ragged tiles + GQA
    (1, 300, 2, 2, 64, False, 0.5),
])
def test_flash_attention_dropout_matches_reference(dph_native, B, S, Hq, Hkv, D, causal, p):
    from distributed_pytorch_hpc_amd.ops.attention import flash_attention

    torch.manual_seed(0)
    dev = "cuda"
    q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    seed = 987654
    scale = 1.0 / math.sqrt(D)
    o = flash_attention(q, k, v, causal=causal, dropout_p=p, seed=seed)
    mask = dropout_mask(B, Hq, S, S, p, seed, device=dev)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _reference(qr, kr, vr, mask, p, causal, scale)
    assert rel_err(o, orf) < 2e-2
    g = torch.randn_like(orf)
    o.backward(g.to(torch.bfloat16))
    orf.backward(g)
    for a, b in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        assert rel_err(a, b) < 3e-2
    # the same seed reproduces the output; p = 0 is the plain kernel
    o2 = flash_attention(q, k, v, causal=causal, dropout_p=p, seed=seed)
    assert torch.equal(o, o2)
