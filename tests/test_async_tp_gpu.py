"""Async-TP micro-GEMMs on the GPU (parallel/async_tp.py): with one sequence per rank the all-gather x GEMM writes
each micro-GEMM's [P, m, N] result straight into its rank-major rows of y through one strided-batched GEMM (batch
stride k m N, broadcast weight); with B > 1 it copies.  A single process simulates the 8-rank all-gather (rank p's
shard = x + p), so y must equal the full gathered sequence @ op(w) in rank-major order -- the layout the
sequence-parallel layers expect -- against an fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

P = 8


class _Done:
    def wait(self):
        pass


def _sim_ag(x, group, out=None):
    """all_gather_into_tensor stand-in: rank p contributes x + p (dim-0 concatenation)."""
    if out is None:
        out = torch.empty((P * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
    for p in range(P):
        out[p * x.shape[0]:(p + 1) * x.shape[0]] = x + p
    return out.view(P, *x.shape), _Done()


@pytest.mark.parametrize("B,k,transpose_w", [(1, 2, True), (1, 4, False), (2, 2, True), (2, 2, False)])
def test_ag_matmul_rank_major_rows(monkeypatch, B, k, transpose_w):
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel import async_tp

    _lib.require()
    monkeypatch.setattr(async_tp, "_ws", lambda group: P)
    monkeypatch.setattr(async_tp, "_ag_async", _sim_ag)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    Sl, D, N = 256, 512, 384
    x = (0.5 * torch.randn(B, Sl, D, device=dev, generator=g)).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, D, device=dev, generator=g)).to(torch.bfloat16) if transpose_w else \
        (0.05 * torch.randn(D, N, device=dev, generator=g)).to(torch.bfloat16)
    y, xg = async_tp._ag_matmul(x, w, None, k, transpose_w)
    full = torch.cat([(x + p).float() for p in range(P)], 1)          # [B, P * Sl, D], rank-major sequence
    ref = full @ (w.t() if transpose_w else w).float()
    assert y.shape == (B, P * Sl, N)
    err = (y.float() - ref).norm() / ref.norm()
    assert err < 5e-3, err
    # the gathered buffer is chunk-major [k, P, B, m, D] (the weight gradient's operand)
    m = Sl // k
    assert torch.equal(xg[1, 3], (x[:, m:2 * m] + 3))


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
