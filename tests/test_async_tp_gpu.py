"""Async-TP on the GPU (parallel/async_tp.py, parallel/fused_layers.py _SwiGLUMLPAsyncFn).  One process simulates the
8-rank collectives (rank p's token shard = x + p; a reduce-scatter returns P x this rank's rows), so the results must
equal the full token matrix in natural order -- round c of the deal, rank p at rows [c P m + p m, +m) -- times the
weights, against fp32 references of the same formulas."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu

P = 8


class _Done:
    def wait(self):
        pass


def _fake_dist():
    def ag(out, x, group=None, async_op=False):
        m = x.shape[0]
        for p in range(P):
            out[p * m:(p + 1) * m] = x + p
        return _Done()

    def rs(out, x, op=None, group=None, async_op=False):
        m = out.shape[0]
        out.copy_(P * x[:m])   # every rank holds the same partial in the simulation; this is rank 0's rows
        return _Done()

    return types.SimpleNamespace(all_gather_into_tensor=ag, reduce_scatter_tensor=rs, get_world_size=lambda g=None: P,
                                 ReduceOp=torch.distributed.ReduceOp)


def _natural(x2, k):
    """Rank p's shard x2 + p dealt in k rounds -> the full [P n, D] token matrix in natural order."""
    n, d = x2.shape
    m = n // k
    return torch.stack([torch.stack([x2[c * m:(c + 1) * m] + p for p in range(P)]) for c in range(k)]).reshape(-1, d)


@pytest.mark.parametrize("k,transpose_w", [(1, True), (2, True), (2, False), (4, False)])
def test_ag_matmul_natural_token_order(monkeypatch, k, transpose_w):
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel import async_tp

    _lib.require()
    monkeypatch.setattr(async_tp, "_ws", lambda group: P)
    monkeypatch.setattr(async_tp, "dist", _fake_dist())
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    n, D, N = 512, 512, 384
    x2 = (0.5 * torch.randn(n, D, device=dev, generator=g)).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, D, device=dev, generator=g)).to(torch.bfloat16) if transpose_w else \
        (0.05 * torch.randn(D, N, device=dev, generator=g)).to(torch.bfloat16)
    y, xg = async_tp._ag_matmul(x2, w, None, k, transpose_w)
    full = _natural(x2.float(), k)
    assert torch.equal(xg.float(), _natural(x2, k).float())   # the weight gradient's operand: natural order
    ref = full @ (w.t() if transpose_w else w).float()
    err = (y.float() - ref).norm() / ref.norm()
    assert y.shape == (P * n, N) and err < 5e-3, err
    # reduce-scatter side: rank 0's rows of every round, P x (the simulated sum)
    w_rs = (0.05 * torch.randn(D, N, device=dev, generator=g)).to(torch.bfloat16)   # y @ w_rs^T: [P n, D]
    ys = async_tp._matmul_rs(y, w_rs, None, k, True)
    part = y.float() @ w_rs.float().t()
    m = n // k
    ref_rs = torch.cat([P * part[c * P * m: c * P * m + m] for c in range(k)])
    assert ys.shape == (n, D) and ((ys.float() - ref_rs).norm() / ref_rs.norm()) < 5e-3


@pytest.mark.parametrize("k", [1, 2])
def test_async_fused_swiglu_mlp_matches_formulas(monkeypatch, k):
    """The fused SwiGLU MLP with pipelined token collectives (async TP keeps the fused kernels): forward and every
    gradient against fp32 references on the simulated 8-rank collectives."""
    import torch.nn.functional as F

    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel import fused_layers

    _lib.require()
    import torch.distributed as real_dist
    fake = _fake_dist()
    monkeypatch.setattr(real_dist, "all_gather_into_tensor", fake.all_gather_into_tensor)
    monkeypatch.setattr(real_dist, "reduce_scatter_tensor", fake.reduce_scatter_tensor)
    monkeypatch.setattr(real_dist, "get_world_size", fake.get_world_size)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    n, D, H = 512, 256, 384        # local tokens, model dim, local hidden
    x = (0.5 * torch.randn(1, n, D, device=dev, generator=g)).to(torch.bfloat16).requires_grad_()
    w13 = (0.05 * torch.randn(2 * H, D, device=dev, generator=g)).to(torch.bfloat16).requires_grad_()
    w2 = (0.05 * torch.randn(D, H, device=dev, generator=g)).to(torch.bfloat16).requires_grad_()
    y = fused_layers._SwiGLUMLPAsyncFn.apply(x, w13, w2, None, k)
    dy = (0.5 * torch.randn(1, n, D, device=dev, generator=g)).to(torch.bfloat16)
    y.backward(dy)
    # fp32 references of the same (simulated) collectives
    m = n // k
    xg = _natural(x.detach()[0].float(), k)
    x13 = xg @ w13.detach().float().t()
    a, u = x13[:, :H], x13[:, H:]
    h = F.silu(a) * u
    part = h @ w2.detach().float().t()
    y_ref = torch.cat([P * part[c * P * m: c * P * m + m] for c in range(k)])
    assert ((y[0].float() - y_ref).norm() / y_ref.norm()) < 2e-2
    dyg = _natural(dy[0].float(), k)
    dh = dyg @ w2.detach().float()
    sa = torch.sigmoid(a)
    d13 = torch.cat([dh * u * (sa * (1 + a * (1 - sa))), dh * F.silu(a)], 1)
    dxp = d13 @ w13.detach().float()
    dx_ref = torch.cat([P * dxp[c * P * m: c * P * m + m] for c in range(k)])
    for got, ref in ((x.grad[0], dx_ref), (w2.grad, dyg.t() @ h), (w13.grad, d13.t() @ xg)):
        assert ((got.float() - ref).norm() / ref.norm()) < 3e-2


def test_dgrad_of_noncontiguous_3d_grad_is_one_2d_gemm(dph_native):
    """The input gradient of a linear layer whose incoming gradient is a non-contiguous 3-D view (the adjoint of a
    sequence-parallel reduce-scatter): folded into one 2-D GEMM (torch.matmul would broadcast the weight at batch
    stride 0, which hipBLASLt on this stack rejects and whose fallback faulted the GPU at the TP = 8 w2 shape)."""
    from distributed_pytorch_hpc_amd.parallel.linear import _dgrad

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    base = torch.randn(1024, 4, 4096, device=dev, generator=g).to(torch.bfloat16)
    gy = base.transpose(0, 1)                                       # [4, 1024, 4096]: leading dims not foldable
    assert not gy.is_contiguous()
    w = (0.02 * torch.randn(4096, 1376, device=dev, generator=g)).to(torch.bfloat16)
    dx = _dgrad(gy, w)
    ref = gy.float() @ w.float()
    assert dx.shape == (4, 1024, 1376)
    assert ((dx.float() - ref).norm() / ref.norm()).item() < 5e-3
