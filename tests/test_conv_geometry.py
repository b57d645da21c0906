"""The gathered implicit-GEMM geometry of the strided convolutions (ops/conv.py conv_geo / strided_fwd_geo /
strided_dgrad_classes), checked on the CPU through its fp32 PyTorch model ``convg_reference`` against
torch.nn.functional.conv2d and its autograd input gradient: the forward's strided source pixels and the input
gradient's parity classes (taps per class, scattered destination rows, zero classes of a 1x1 stride-2)."""
import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_hpc_amd.ops.conv import (convg_reference, strided_dgrad_classes, strided_dgrad_covers_all,
                                                  strided_fwd_geo, strided_out_hw)


@pytest.mark.parametrize("H,W,k,s,p", [(8, 8, 3, 2, 1), (7, 7, 3, 2, 1), (9, 6, 3, 2, 1), (8, 8, 1, 2, 0),
                                       (7, 5, 1, 2, 0), (10, 10, 3, 3, 1)])
def test_strided_geometry_matches_conv2d(H, W, k, s, p):
    torch.manual_seed(0)
    B, C, Co = 2, 4, 6
    x = torch.randn(B, C, H, W, requires_grad=True)
    w = torch.randn(Co, C, k, k)
    y = F.conv2d(x, w, stride=s, padding=p)
    Ho, Wo = strided_out_hw(H, W, k, s, p)
    x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, C)
    wk = w.permute(0, 2, 3, 1).reshape(Co, k * k * C)
    y2 = convg_reference(x2, wk, strided_fwd_geo(H, W, k, s, p))
    assert torch.allclose(y2.view(B, Ho, Wo, Co).permute(0, 3, 1, 2), y, atol=1e-4)
    dy = torch.randn_like(y)
    y.backward(dy)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, Co)
    dx2 = torch.zeros(B * H * W, C)
    wp = w.permute(1, 2, 3, 0)
    covered = 0
    for geo, kt in strided_dgrad_classes(H, W, k, s, p):
        covered += geo[2] * geo[3]
        bk = torch.stack([wp[:, ky, kx, :] for ky, kx in kt], 1).reshape(C, len(kt) * Co)
        convg_reference(dy2, bk, geo, dx2)
    assert torch.allclose(dx2.view(B, H, W, C).permute(0, 3, 1, 2), x.grad, atol=1e-4)
    assert strided_dgrad_covers_all(H, W, k, s, p) == (covered == H * W)
    assert strided_dgrad_covers_all(H, W, k, s, p) == (k >= s)


def _chunk_tap_gather(a, geo, B):
    """[B * Hp * Wq, 8] pair-pixel rows -> the stem GEMM's gathered operand [B * Ho * Wo, ntaps * 8]."""
    Hp, Wq, Ho, Wo, nt, kxp = geo[0], geo[1], geo[2], geo[3], geo[14], geo[24]
    img = a.view(B, Hp, Wq, 8)
    cols = []
    for t in range(nt):
        ty, tx = t // kxp, t % kxp
        cols.append(img[:, 2 * torch.arange(Ho)[:, None] + ty, torch.arange(Wo)[None, :] + tx])
    return torch.cat(cols, -1).reshape(B * Ho * Wo, nt * 8)


@pytest.mark.parametrize("H,W,k,p", [(16, 16, 7, 3), (15, 12, 7, 3), (10, 10, 5, 2), (9, 9, 3, 1)])
def test_stem_chunk_tap_layout(H, W, k, p):
    """The RGB stem as a chunk-tap GEMM (ops/conv.py stem_geometry / stem_weight): forward and weight gradient through
    the pair-pixel gather equal F.conv2d and its weight gradient; the weight-gradient columns fold back to [Cout,3,k,k]."""
    from distributed_pytorch_hpc_amd.ops.conv import stem_geometry, stem_weight

    torch.manual_seed(1)
    B, C, Co = 2, 3, 8
    x = torch.randn(B, C, H, W)
    w = torch.randn(Co, C, k, k, requires_grad=True)
    y = F.conv2d(x, w, stride=2, padding=p)
    Hp, Wq, Ho, Wo, kxp, nt, K, geo = stem_geometry(H, W, k, p)
    assert (Ho, Wo) == tuple(y.shape[2:]) and K % 128 == 0 and K >= nt * 8
    xp = torch.zeros(B, Hp, 2 * Wq, 4)
    xp[:, p:p + H, p:p + W, :C] = x.permute(0, 2, 3, 1)
    g = _chunk_tap_gather(xp.view(B * Hp * Wq, 8), geo, B)
    wk = stem_weight(w.detach(), kxp, K)
    y2 = g @ wk[:, :nt * 8].t()
    assert torch.allclose(y2.view(B, Ho, Wo, Co).permute(0, 3, 1, 2), y, atol=1e-4)
    dy = torch.randn_like(y)
    y.backward(dy)
    gk = torch.zeros(Co, K)
    gk[:, :nt * 8] = dy.permute(0, 2, 3, 1).reshape(-1, Co).t() @ g
    g5 = gk[:, :k * kxp * 8].view(Co, k, kxp, 2, 4).permute(0, 4, 1, 2, 3).reshape(Co, 4, k, 2 * kxp)
    assert torch.allclose(g5[:, :C, :, :k], w.grad, atol=1e-3)
