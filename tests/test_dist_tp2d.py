"""2-D tensor parallelism (doc-only in the reference, docs/guide/06_tensor_parallel.md:105-128): a (2 x 2) grid
and a (1 x 2) / (2 x 1) degenerate grid must reproduce the single-process forward, loss and every parameter
gradient of the same MLP block (LayerNorm -> Linear -> GELU -> Linear -> RMSNorm), gloo on CPU."""
import pytest
import torch
from torch import nn

from dist_utils import run_distributed


def _model():
    from distributed_pytorch_hpc_amd import ops

    torch.manual_seed(3)
    return nn.Sequential(nn.LayerNorm(32), nn.Linear(32, 64), nn.GELU(), nn.Linear(64, 32, bias=False),
                         ops.RMSNorm(32, eps=1e-5))


def _data():
    g = torch.Generator().manual_seed(11)
    return torch.randn(2, 8, 32, generator=g), torch.randn(2, 8, 32, generator=g)


def _reference():
    m = _model()
    x, y = _data()
    loss = (m(x) - y).pow(2).mean()
    loss.backward()
    return loss.detach(), m(x).detach(), {n: p.grad.clone() for n, p in m.named_parameters()}


def _worker(rank, world, rows, cols):
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel_2d import (Grid2D, gather_activation_2d, mse_loss_2d,
                                                                         parallelize_2d, shard_activation_2d)

    grid = Grid2D(rows, cols)
    m = parallelize_2d(_model(), grid)
    x, y = _data()
    xs, ys = shard_activation_2d(x, grid), shard_activation_2d(y, grid)
    out = m(xs)
    local, tot = mse_loss_2d(out, ys, grid)
    local.backward()
    full = gather_activation_2d(out.detach(), grid)
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    return {"loss": tot, "out": full, "grads": grads, "i": grid.i, "j": grid.j}


def _full_grad_block(g_full, name, shape_local, rows, cols, i, j):
    """The block of a full-model gradient that rank (i, j) owns."""
    if g_full.dim() == 2:      # Linear2D weight [N_j, K_i]
        return g_full.chunk(cols, 0)[j].chunk(rows, 1)[i]
    return g_full.chunk(cols, 0)[j]


@pytest.mark.parametrize("rows,cols", [(2, 2), (1, 2), (2, 1)])
def test_tp2d_matches_single_process(rows, cols):
    ref_loss, ref_out, ref_grads = _reference()
    res = run_distributed(_worker, rows * cols, rows, cols)
    for r in res:
        assert torch.allclose(r["loss"], ref_loss, atol=1e-6, rtol=1e-5)
        assert torch.allclose(r["out"], ref_out, atol=1e-5, rtol=1e-4)
        for n, g in r["grads"].items():
            exp = _full_grad_block(ref_grads[n], n, g.shape, rows, cols, r["i"], r["j"])
            assert exp.shape == g.shape, (n, exp.shape, g.shape)
            assert torch.allclose(g, exp, atol=1e-5, rtol=1e-4), (n, (g - exp).abs().max())
