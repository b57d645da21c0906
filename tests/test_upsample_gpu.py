"""UNet up-path kernels (csrc/upsample.hip, ops/upsample.py) vs the fp32 PyTorch reference sequence
ConvTranspose2d(2, 2) -> bilinear resize -> cat (multinode_ddp_unet.py:180-188, 205-213)."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


def _need():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


# (N, Cin, Co, H, W, Cs, Ho, Wo): the three ERA5 decoder levels of SimpleUNet(65, 65, 64) at 181 x 360, plus odd
# ratios (down-sizing back to < 2H, a resize along both axes)
SHAPES = [
    (2, 512, 256, 22, 45, 256, 45, 90),     # up3: 44 -> 45 rows
    (2, 256, 128, 45, 90, 128, 90, 180),    # up2: no resize
    (1, 128, 64, 90, 180, 64, 181, 360),    # up1: 180 -> 181 rows
    (2, 64, 32, 7, 9, 16, 11, 21),          # resize on both axes (ratios 14/11, 18/21)
    (1, 32, 16, 5, 6, 8, 17, 23),           # up-sizing beyond 2x of the transposed output
]


@pytest.mark.parametrize("shape", SHAPES)
def test_up_concat_matches_fp32_reference(shape):
    _need()
    from distributed_pytorch_hpc_amd.ops.upsample import up_concat, up_concat_native_ok, up_concat_reference

    n, cin, co, h, w, cs, ho, wo = shape
    dev = torch.device("cuda")
    torch.manual_seed(0)
    up = nn.ConvTranspose2d(cin, co, 2, 2).to(dev)
    x = _cl(torch.randn(n, cin, h, w, device=dev)).bfloat16()
    skip = _cl(torch.randn(n, cs, ho, wo, device=dev)).bfloat16()
    up_b = nn.ConvTranspose2d(cin, co, 2, 2).to(dev).bfloat16()
    up_b.load_state_dict({k: v.bfloat16() for k, v in up.state_dict().items()})
    assert up_concat_native_ok(up_b, x, skip)

    xr = x.float().requires_grad_(True)
    sr = skip.float().requires_grad_(True)
    ref = up_concat_reference(up, xr, sr)
    xb, sb = x.clone().requires_grad_(True), skip.clone().requires_grad_(True)
    out = up_concat(up_b, xb, sb)
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    err = (out.float() - ref).abs().max().item()
    assert err < 3e-2 * ref.abs().max().item(), err
    assert torch.equal(out[:, co:], skip)                       # the skip half is an exact copy

    g = _cl(torch.randn_like(ref))
    ref.backward(g)
    out.backward(g.bfloat16())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

    assert rel(xb.grad, xr.grad) < 2e-2
    assert torch.equal(sb.grad, g[:, co:].bfloat16())
    assert rel(up_b.weight.grad, up.weight.grad) < 2e-2
    assert rel(up_b.bias.grad, up.bias.grad) < 1e-2


def test_up_concat_adjoint_exact_fp32():
    """fp32 through the kernels: the backward is the exact adjoint of the forward (<dcat, F(x)> = <F^T dcat, x>)."""
    _need()
    from distributed_pytorch_hpc_amd.ops import _lib

    dev = torch.device("cuda")
    n, co, h, w, cs, ho, wo = 2, 16, 9, 11, 8, 19, 23
    y2 = torch.randn(n * h * w, 4 * co, device=dev)
    skip = _cl(torch.randn(n, cs, ho, wo, device=dev))
    out = _lib.ops().upcat_fwd(y2, None, skip, h, w)
    dcat = _cl(torch.randn_like(out))
    dy2, dskip = _lib.ops().upcat_bwd(dcat, h, w, co)
    lhs = (dcat[:, :co].double() * out[:, :co].double()).sum()
    rhs = (dy2.double() * y2.double()).sum()
    assert abs(lhs - rhs).item() < 1e-4 * abs(lhs).item()
    assert torch.equal(dskip, dcat[:, co:].contiguous(memory_format=torch.channels_last))


def test_unet_fused_up_path_step_matches_reference():
    """SimpleUNet forward + backward under bf16 autocast: fused up-path vs the three-op sequence (transposed conv,
    ATen bilinear, cat), every other op on the same native kernels.  (The all-ATen reference mode is not used
    here: MIOpen's batch norm on bf16 channels-last autocast input crashed the process on the test box.)"""
    _need()
    from distributed_pytorch_hpc_amd.models.unet import SimpleUNet, to_channels_last
    from distributed_pytorch_hpc_amd.ops import upsample
    from distributed_pytorch_hpc_amd.ops.loss import latitude_weighted_mse

    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = to_channels_last(SimpleUNet(16, 16, 32).to(dev))
    x = _cl(torch.randn(2, 16, 45, 90, device=dev))
    y = _cl(torch.randn(2, 16, 45, 90, device=dev))

    def run(fused, amp=True):
        m.zero_grad(set_to_none=True)
        old = upsample.up_concat_native_ok
        if not fused:   # the reference three-op sequence
            upsample.up_concat_native_ok = lambda *a: False
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out = m(x)
            loss = latitude_weighted_mse(out.float(), y)
            loss.backward()
        finally:
            upsample.up_concat_native_ok = old
        return loss.item(), {k: p.grad.float().clone() for k, p in m.named_parameters()}

    l32, g32 = run(False, amp=False)           # fp32 everywhere: the yardstick for both bf16 paths
    l_ref, g_ref = run(False)
    l_dph, g_dph = run(True)
    assert abs(l_ref - l_dph) < 1e-2 * abs(l_ref) and abs(l32 - l_dph) < 2e-2 * abs(l32)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    for k in ("up3.weight", "up3.bias", "up2.weight", "up2.bias", "up1.weight", "up1.bias", "dec1.0.weight",
              "enc1.0.weight"):
        e_dph, e_ref = rel(g_dph[k], g32[k]), rel(g_ref[k], g32[k])
        # the fused bf16 path is no further from fp32 than the unfused bf16 path (plus a small margin)
        assert e_dph < 1.5 * e_ref + 2e-2, (k, e_dph, e_ref)
