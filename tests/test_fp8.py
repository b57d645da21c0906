"""Opt-in FP8-GEMM mode (ops/fp8.py, csrc/fp8.hip) against fp32 / bf16 references (GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("fmt,dt,fmax", [(0, torch.float8_e4m3fn, 448.0), (1, torch.float8_e5m2, 57344.0)])
@pytest.mark.parametrize("R,C", [(256, 192), (64, 4096), (1024, 1088)])
def test_quantize_matches_torch_cast(dph_native, fmt, dt, fmax, R, C):
    """Row-major and transposed copies equal torch's own cast of x * FMAX / amax (bitwise, RNE), dequant = amax/FMAX."""
    from distributed_pytorch_hpc_amd.ops import fp8

    torch.manual_seed(fmt * 7 + R)
    x = (torch.randn(R, C, device=DEV) * 3).to(torch.bfloat16)
    x[3, 5] = -17.5                                            # a known amax
    y, yt, s = fp8.quantize(x, fmt, rowmajor=True, transposed=True)
    amax = x.float().abs().max()
    ref = (x.float() * (fmax / amax)).clamp(-fmax, fmax).to(dt)
    assert y.dtype == dt and yt.shape == (C, R)
    assert torch.equal(y.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(yt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert abs(s.item() - amax.item() / fmax) <= 1e-6 * amax.item()


def test_fp8_linear_fwd_bwd_close_to_fp32(dph_native):
    from distributed_pytorch_hpc_amd.ops import fp8

    torch.manual_seed(3)
    x = torch.randn(4, 64, 512, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(768, 512, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    fp8.set_fp8(True)
    try:
        y = fp8.fp8_linear(x, w)
    finally:
        fp8.set_fp8(False)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    yr = xr @ wr.t()
    yr.backward(g.float())
    assert rel_err(y, yr) < 4e-2
    assert rel_err(x.grad, xr.grad) < 6e-2 and rel_err(w.grad, wr.grad) < 6e-2


def test_fp8_llama_training_tracks_bf16(dph_native):
    """A tiny Llama under the data-parallel engine: fp8 GEMM losses track the bf16 run and still decrease."""
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.ops import fp8
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    args = ModelArgs(dim=512, n_layers=2, n_heads=8, vocab_size=1024, max_seq_len=256)
    g = torch.Generator(device=DEV).manual_seed(0)
    data = [torch.randint(0, 64, (4, 257), device=DEV, generator=g) for _ in range(2)]   # learnable: 64 tokens

    def run(use_fp8):
        model = build_llama(args, device=DEV, dtype=torch.bfloat16, seed=1)
        if use_fp8:
            fp8.enable_for_llama(model)
        eng = DataParallelEngine(model)
        eng.configure_optimizer(OptimConfig(lr=1e-3))
        losses = []
        try:
            for i in range(12):
                t = data[i % 2]
                loss = model(t[:, :-1], t[:, 1:])
                loss.backward()
                eng.step()
                eng.zero_grad()
                losses.append(loss.item())
        finally:
            fp8.set_fp8(False)
        return losses

    ref, got = run(False), run(True)
    assert got[-1] < got[0] - 0.5, got
    assert all(abs(a - b) < 0.05 * abs(b) + 0.05 for a, b in zip(got, ref)), (got, ref)
