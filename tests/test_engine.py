"""Single-process checks of the data-parallel engine's fast paths against stock PyTorch."""
import pytest
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


def test_channels_last_weights_stay_channels_last_in_flat_buckets():
    """utils.flat.param_view: channels-last conv weights become channels-last views of the engine's flat buffer
    (no per-call NHWC copies for MIOpen); values and SGD updates match a plain-layout copy of the model."""
    import torch.nn.functional as F

    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, padding=1, bias=False), torch.nn.ReLU(),
                              torch.nn.Conv2d(8, 4, 3, padding=1))
    cl = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, padding=1, bias=False), torch.nn.ReLU(),
                             torch.nn.Conv2d(8, 4, 3, padding=1))
    cl.load_state_dict(ref.state_dict())
    cl = cl.to(memory_format=torch.channels_last)
    engines = [DataParallelEngine(m) for m in (ref, cl)]
    for e in engines:
        e.configure_optimizer(OptimConfig("sgd", lr=0.1, momentum=0.9))
    w = cl[0].weight
    assert w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
    assert w.main_grad.is_contiguous(memory_format=torch.channels_last)
    assert w.untyped_storage().data_ptr() == engines[1].flat_param.untyped_storage().data_ptr()
    x = torch.randn(2, 4, 6, 6)
    for _ in range(2):
        for m, e in zip((ref, cl), engines):
            e.zero_grad()
            F.mse_loss(m(x.contiguous(memory_format=torch.channels_last) if m is cl else x), x).backward()
            e.step()
    for a, b in zip(ref.parameters(), cl.parameters()):
        assert torch.allclose(a, b, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["adamw", "sgd"])
def test_overlapped_optimizer_step_matches_inline(dph_native, name):
    """The optimizer update on a side stream (waited for per module by the next forward) gives bit-identical
    parameters to the update on the compute stream, step after step, including a parameter the forward never uses
    (its bucket is only covered by the root-forward join) and with gradient clipping."""
    from distributed_pytorch_hpc_amd.models.llama2 import build_llama
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    def run(overlap):
        m = build_llama("tiny", device="cuda", seed=3)
        m.unused = torch.nn.Parameter(torch.randn(64, device="cuda", dtype=torch.bfloat16))
        eng = DataParallelEngine(m, bucket_cap_mb=0.05, overlap_step=overlap)   # explicit: the default is off
        eng.configure_optimizer(OptimConfig(name, lr=1e-3, momentum=0.9, weight_decay=0.1,
                                            max_grad_norm=1.0 if name == "adamw" else None))
        g = torch.Generator(device="cuda").manual_seed(0)
        losses = []
        for _ in range(5):
            t = torch.randint(0, 512, (2, 129), device="cuda", generator=g)
            loss = m(t[:, :-1], t[:, 1:])
            loss.backward()
            eng.step()
            eng.zero_grad()
            # unrelated work on the compute stream between steps must not see stale parameters
            junk = torch.full((1 << 22,), float("nan"), device="cuda")
            del junk
            losses.append(loss.detach())
        eng.synchronize()
        torch.cuda.synchronize()
        assert (eng._opt_stream is not None) == overlap
        return [p.detach().clone() for p in m.parameters()], torch.stack(losses)

    pa, la = run(True)
    pb, lb = run(False)
    assert torch.equal(la, lb)
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)


def test_fp8_mode_falls_back_off_gpu():
    """FP8 GEMM mode (ops/fp8.py) only engages on bf16 CUDA tensors: on CPU the step is the plain one, bit for bit."""
    import torch

    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.ops import fp8
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    args = ModelArgs(dim=64, n_layers=1, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)
    t = torch.randint(0, 128, (2, 33), generator=torch.Generator().manual_seed(0))

    def run(on):
        m = build_llama(args, device="cpu", dtype=torch.float32, seed=2)
        if on:
            fp8.enable_for_llama(m)
        eng = DataParallelEngine(m)
        eng.configure_optimizer(OptimConfig(lr=1e-2))
        try:
            loss = m(t[:, :-1], t[:, 1:])
            loss.backward()
            eng.step()
        finally:
            fp8.set_fp8(False)
        return loss.item(), [p.detach().clone() for p in m.parameters()]

    (l0, p0), (l1, p1) = run(False), run(True)
    assert l0 == l1 and all(torch.equal(a, b) for a, b in zip(p0, p1))


def test_fp8_exemption_survives_tp_sharding():
    """The LM head is FP8-exempt by construction, and the marker is carried onto its tensor-parallel shard."""
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, Transformer
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import ColwiseParallelLinear, RowwiseParallelLinear

    m = Transformer(ModelArgs(dim=64, n_layers=1, n_heads=4, vocab_size=128, multiple_of=32, max_seq_len=16))
    assert getattr(m.output.weight, "_dph_fp8_exempt", False)
    assert not getattr(m.layers[0].attention.wqkv.weight, "_dph_fp8_exempt", False)
    col = ColwiseParallelLinear(m.output, None)
    row = RowwiseParallelLinear(m.output, None)
    assert col.weight._dph_fp8_exempt and row.weight._dph_fp8_exempt
