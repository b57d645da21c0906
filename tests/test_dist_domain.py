"""Domain parallelism: a conv-BN-ReLU stack on a latitude-sharded field equals the unsharded model (gloo)."""

import pytest
import torch
import torch.distributed as dist
from torch import nn

from dist_utils import run_distributed


def _net():
    torch.manual_seed(4)
    return nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(),
                         nn.Conv2d(8, 8, 5, padding=2), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 2, 1))


def _x():
    g = torch.Generator().manual_seed(2)
    return torch.randn(2, 3, 24, 10, generator=g)


def _worker(rank, world):
    from distributed_pytorch_hpc_amd.parallel.domain import convert_to_domain_parallel

    net = convert_to_domain_parallel(_net(), dist.group.WORLD, dim=2)
    x = _x().chunk(world, 2)[rank].clone().requires_grad_()
    y = net(x)
    y.pow(2).sum().backward()
    return y.detach(), x.grad, net[0].conv.weight.grad


@pytest.mark.parametrize("world", [2, 4])
def test_halo_conv_stack_matches_full_field(world):
    net = _net()
    x = _x().requires_grad_()
    y = net(x)
    y.pow(2).sum().backward()
    outs = run_distributed(_worker, world)
    ys = torch.cat([o[0] for o in outs], 2)
    gx = torch.cat([o[1] for o in outs], 2)
    assert torch.allclose(ys, y.detach(), atol=1e-5)
    assert torch.allclose(gx, x.grad, atol=1e-5)
    gw = sum(o[2] for o in outs)
    assert torch.allclose(gw, net[0].weight.grad, atol=1e-4)


def test_single_rank_halo_is_zero_padding():
    from distributed_pytorch_hpc_amd.parallel.domain import halo_exchange

    x = torch.randn(1, 1, 4, 3)
    y = halo_exchange(x, 2, 2, None) if not dist.is_initialized() else None
    assert y.shape == (1, 1, 8, 3) and torch.equal(y[:, :, 2:6], x) and y[:, :, :2].abs().sum() == 0
