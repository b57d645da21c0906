"""Strided convolutions on the gathered implicit-GEMM kernels (ops/conv.py StridedConv2d: csrc/conv3x3.hip conv3_k
GEN forward and parity-class input gradient, csrc/conv1x1.hip c3w_k GEN weight gradient) against F.conv2d in fp32:
ResNet's stride-2 3x3 conv2 and stride-2 1x1 downsample, odd and non-square images, ragged row tiles, the BatchNorm
statistics epilogue, the engine's direct main_grad write, and a downsample bottleneck end to end."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _strided_on(monkeypatch):
    monkeypatch.setenv("DPH_CONV", "dph")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("k,B,C,Co,H,W", [(3, 2, 64, 64, 16, 16), (3, 2, 128, 128, 15, 15), (3, 1, 64, 192, 9, 14),
                                          (3, 3, 256, 256, 14, 14), (1, 2, 256, 512, 14, 14), (1, 2, 64, 128, 7, 9),
                                          (1, 1, 512, 1024, 28, 28)])
@pytest.mark.parametrize("autocast", [False, True])
def test_strided_conv_matches_conv2d(dph_native, k, B, C, Co, H, W, autocast):
    from distributed_pytorch_hpc_amd.ops.conv import StridedConv2d, strided_native_ok

    torch.manual_seed(7)
    p = k // 2
    conv = StridedConv2d(C, Co, k, 2, p, bias=False).to(DEV).to(memory_format=torch.channels_last)
    if not autocast:
        conv = conv.to(torch.bfloat16)
    x = torch.randn(B, C, H, W, device=DEV, dtype=torch.float32 if autocast else torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        assert strided_native_ok(x, conv)
        y = conv(x)
    g = torch.randn_like(y.float())
    y.float().backward(g)
    xr = x.detach().to(torch.bfloat16).float().requires_grad_()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, wr, stride=2, padding=p)
    yr.backward(g)
    assert y.shape == yr.shape
    assert rel_err(y, yr) < 8e-3
    assert rel_err(x.grad, xr.grad) < 1e-2
    assert rel_err(conv.weight.grad, wr.grad) < 1e-2


def test_strided_conv_stats_epilogue_and_main_grad(dph_native, monkeypatch):
    """The BatchNorm partials from the strided forward equal the output's own statistics; with an engine-owned
    channels-last main_grad the weight-gradient kernel writes (then accumulates) into it directly."""
    from distributed_pytorch_hpc_amd.ops.conv import StatsSlot, StridedConv2d

    torch.manual_seed(3)
    conv = StridedConv2d(128, 128, 3, 2, 1, bias=False).to(DEV).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    x = torch.randn(4, 128, 28, 28, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    slot = StatsSlot()
    y = conv(x, stats_slot=slot)
    y2 = y.permute(0, 2, 3, 1).reshape(-1, 128).float()
    nmb = (y2.shape[0] + 127) // 128
    st = slot.stats
    assert st is not None and st.numel() == 2 * nmb * 128 + nmb
    rows = st[2 * nmb * 128:]
    mean = (st[:nmb * 128].view(nmb, 128) * rows[:, None]).sum(0) / rows.sum()
    assert rel_err(mean, y2.mean(0)) < 1e-3

    w = conv.weight
    w.main_grad = torch.zeros_like(w, dtype=torch.float32).contiguous(memory_format=torch.channels_last)
    calls = []
    w._dph_grad_ready = lambda: calls.append(1)
    w._dph_accum = False
    xg = x.detach().requires_grad_()
    g = torch.randn(4, 128, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for _ in range(2):
        conv(xg).backward(g)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    torch.nn.functional.conv2d(xr, wr, stride=2, padding=1).backward(g.float())
    assert len(calls) == 2 and w.grad is None
    assert rel_err(w.main_grad, 2 * wr.grad) < 1e-2


def test_downsample_bottleneck_strided_path_matches_miopen(dph_native, monkeypatch):
    """A stride-2 ResNet bottleneck (3x3 conv2 and 1x1 downsample strided, bf16 channels-last): input and parameter
    gradients on the gathered kernels match the MIOpen path."""
    from distributed_pytorch_hpc_amd.models.resnet import Bottleneck, conv1x1
    from distributed_pytorch_hpc_amd.ops.batchnorm import BatchNormAct2d

    torch.manual_seed(0)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    block = Bottleneck(256, 128, 2, down).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 28, 28, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()

    def run(flag):
        monkeypatch.setenv("DPH_CONV", flag)
        block.zero_grad(set_to_none=True)
        x.grad = None
        y = block(x)
        y.float().pow(2).mean().backward()
        return y.float().clone(), x.grad.float().clone(), {n: p.grad.float().clone() for n, p in block.named_parameters()}

    y1, gx1, g1 = run("dph")
    y0, gx0, g0 = run("miopen")
    assert rel_err(y1, y0) < 2e-2
    assert rel_err(gx1, gx0) < 3e-2
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 5e-2, n


@pytest.mark.parametrize("n,H,W,K,N", [(2, 14, 14, 128, 256), (1, 7, 9, 64, 128), (3, 28, 28, 256, 64)])
def test_ts_gemm_nt_add_sub(dph_native, n, H, W, K, N):
    """1x1 dgrad + a stride-2 sub-image gradient added at the even pixels (the strided downsample's hand-off)."""
    torch.manual_seed(n * H + W)
    a = torch.randn(n * H * W, K, device=DEV, dtype=torch.bfloat16)
    b = (0.1 * torch.randn(N, K, device=DEV)).to(torch.bfloat16)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    d = torch.randn(n * Ho * Wo, N, device=DEV, dtype=torch.bfloat16)
    c = torch.ops.dph.ts_gemm_nt_add_sub(a, b, d, H, W, 2)
    ref = (a.float() @ b.float().t()).view(n, H, W, N)
    ref[:, ::2, ::2] += d.float().view(n, Ho, Wo, N)
    assert rel_err(c, ref.view(-1, N)) < 5e-3


def test_downsample_hands_sub_gradient_to_conv1(dph_native, monkeypatch):
    """The strided 1x1 downsample parks its sub-image gradient in conv1's GradSlot (no full-size dX of its own)."""
    import importlib

    from distributed_pytorch_hpc_amd.ops.conv import GradSlot

    resnet_mod = importlib.import_module("distributed_pytorch_hpc_amd.models.resnet")
    made = []

    class _Spy(GradSlot):
        __slots__ = ()

        def __init__(self):
            super().__init__()
            made.append(self)

    monkeypatch.setattr(resnet_mod, "GradSlot", _Spy)
    torch.manual_seed(1)
    down = torch.nn.Sequential(resnet_mod.conv1x1(256, 512, 2),
                               resnet_mod.BatchNormAct2d(512, act=False))
    block = resnet_mod.Bottleneck(256, 128, 2, down).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(2, 256, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    block(x).float().pow(2).mean().backward()
    assert made and made[0].armed and made[0].sub == (2, 14, 14) and made[0].t is None
    assert x.grad is not None and torch.isfinite(x.grad.float()).all()


@pytest.mark.parametrize("B,H,W,Co,k,p", [(2, 224, 224, 64, 7, 3), (3, 37, 50, 64, 7, 3), (2, 32, 32, 128, 5, 2)])
@pytest.mark.parametrize("autocast", [False, True])
def test_stem_conv_matches_conv2d(dph_native, B, H, W, Co, k, p, autocast):
    """The RGB stem on the chunk-tap implicit GEMM (forward + weight gradient) vs F.conv2d in fp32, with the
    following BatchNorm's statistics from the epilogue."""
    from distributed_pytorch_hpc_amd.ops.conv import StatsSlot, StemConv2d, stem_native_ok

    torch.manual_seed(2)
    conv = StemConv2d(3, Co, k, 2, p, bias=False).to(DEV).to(memory_format=torch.channels_last)
    if not autocast:
        conv = conv.to(torch.bfloat16)
    x = torch.randn(B, 3, H, W, device=DEV, dtype=torch.float32 if autocast else torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    slot = StatsSlot()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        assert stem_native_ok(x, conv)
        y = conv(x, stats_slot=slot)
    g = torch.randn_like(y.float())
    y.float().backward(g)
    xr = x.detach().to(torch.bfloat16).float()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, wr, stride=2, padding=p)
    yr.backward(g)
    assert y.shape == yr.shape
    assert rel_err(y, yr) < 8e-3
    assert rel_err(conv.weight.grad, wr.grad) < 1e-2
    y2 = y.permute(0, 2, 3, 1).reshape(-1, Co).float()
    nmb = (y2.shape[0] + 127) // 128
    st = slot.stats
    rows = st[2 * nmb * Co:]
    mean = (st[:nmb * Co].view(nmb, Co) * rows[:, None]).sum(0) / rows.sum()
    assert rel_err(mean, y2.mean(0)) < 1e-3
