"""Single-process checks of the data-parallel engine's fast paths against stock PyTorch."""
import torch
from torch import nn

from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig


def _pair():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 4))
    ref = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 4))
    ref.load_state_dict(m.state_dict())
    return m, ref


def test_main_grad_linear_matches_autograd_fp32():
    m, ref = _pair()
    DataParallelEngine(m).configure_optimizer(OptimConfig("sgd", lr=0.1, weight_decay=0.0))
    x = torch.randn(8, 16)
    m(x).pow(2).sum().backward()
    ref(x).pow(2).sum().backward()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a.main_grad, b.grad)


def test_main_grad_linear_under_autocast_bf16():
    """autocast inputs reach the custom linear in bf16 while parameters stay fp32 (ResNet/UNet --amp)."""
    m, ref = _pair()
    DataParallelEngine(m).configure_optimizer(OptimConfig("sgd", lr=0.1, weight_decay=0.0))
    x = torch.randn(8, 16)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        y, yr = m(x), ref(x)
    assert y.dtype == yr.dtype == torch.bfloat16
    y.float().sum().backward()
    yr.float().sum().backward()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a.main_grad, b.grad)


def test_gradient_accumulation_two_microbatches():
    m, ref = _pair()
    eng = DataParallelEngine(m)
    eng.configure_optimizer(OptimConfig("sgd", lr=0.1, weight_decay=0.0))
    xs = torch.randn(2, 8, 16)
    with eng.no_sync():
        m(xs[0]).sum().backward()
    m(xs[1]).sum().backward()
    ref(xs[0]).sum().backward()
    ref(xs[1]).sum().backward()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a.main_grad, b.grad)
