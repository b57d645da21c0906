"""gloo parity of Ulysses and ring attention (and their Llama integration) against full-sequence attention."""
import math

import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed


def _qkv(b=2, s=32, h=4, d=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(b, s, h, d, generator=g) for _ in range(3)]


def _ring_worker(rank, world, causal):
    from distributed_pytorch_hpc_amd.parallel.context_parallel import ring_attention

    q, k, v = _qkv()
    sl = slice(rank * q.shape[1] // world, (rank + 1) * q.shape[1] // world)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    o = ring_attention(ql, kl, vl, dist.group.WORLD, causal=causal)
    g = torch.Generator().manual_seed(9)
    do = torch.randn(o.shape[0], q.shape[1], *o.shape[2:], generator=g)[:, sl]
    o.backward(do)
    return o.detach(), ql.grad, kl.grad, vl.grad


@pytest.mark.parametrize("world,causal", [(2, True), (4, True), (2, False)])
def test_ring_attention_matches_full(world, causal):
    from distributed_pytorch_hpc_amd.ops.attention import attention_reference

    q, k, v = (t.clone().requires_grad_() for t in _qkv())
    o = attention_reference(q, k, v, causal, 1 / math.sqrt(q.shape[-1]))
    g = torch.Generator().manual_seed(9)
    do = torch.randn(o.shape, generator=g)
    o.backward(do)
    outs = run_distributed(_ring_worker, world, causal)
    S = q.shape[1]
    for r, (ol, dq, dk, dv) in enumerate(outs):
        sl = slice(r * S // world, (r + 1) * S // world)
        assert torch.allclose(ol, o[:, sl].detach(), atol=1e-5)
        assert torch.allclose(dq, q.grad[:, sl], atol=1e-5)
        assert torch.allclose(dk, k.grad[:, sl], atol=1e-5)
        assert torch.allclose(dv, v.grad[:, sl], atol=1e-5)


PRESET = dict(dim=64, n_layers=2, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)


def _llama_worker(rank, world, mode):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.parallel.context_parallel import apply_context_parallel

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=3)
    apply_context_parallel(m, dist.group.WORLD, mode)
    g = torch.Generator().manual_seed(1)
    t = torch.randint(0, 128, (2, 33), generator=g)
    x, y = t[:, :-1], t[:, 1:]
    s = x.shape[1] // world
    loss = m(x[:, rank * s:(rank + 1) * s], y[:, rank * s:(rank + 1) * s])
    loss.backward()
    gw = m.layers[0].attention.wqkv.weight.grad.clone()
    dist.all_reduce(gw)
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    return lt.item() / world, gw / world


@pytest.mark.parametrize("mode", ["ulysses", "ring"])
def test_llama_context_parallel(mode):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=3)
    g = torch.Generator().manual_seed(1)
    t = torch.randint(0, 128, (2, 33), generator=g)
    loss = m(t[:, :-1], t[:, 1:])
    loss.backward()
    ref_g = m.layers[0].attention.wqkv.weight.grad
    outs = run_distributed(_llama_worker, 2, mode)
    for l, gw in outs:
        assert abs(l - loss.item()) < 1e-5
        assert torch.allclose(gw, ref_g, atol=1e-5, rtol=1e-4)


def _zigzag_worker(rank, world):
    from distributed_pytorch_hpc_amd.parallel.context_parallel import ring_attention, shard_sequence

    q, k, v = _qkv(s=48)
    g = torch.Generator().manual_seed(9)
    do = torch.randn(q.shape, generator=g)
    grp = dist.group.WORLD
    ql, kl, vl = (shard_sequence(t, grp, "zigzag").requires_grad_() for t in (q, k, v))
    o = ring_attention(ql, kl, vl, grp, causal=True, layout="zigzag")
    o.backward(shard_sequence(do, grp, "zigzag"))
    return o.detach(), ql.grad, kl.grad, vl.grad


@pytest.mark.parametrize("world", [2, 3])
def test_zigzag_ring_attention_matches_full(world):
    """Load-balanced causal layout: rank r holds chunks r and 2P-1-r."""
    from distributed_pytorch_hpc_amd.ops.attention import attention_reference
    from distributed_pytorch_hpc_amd.parallel.context_parallel import unshard_sequence

    q, k, v = (t.clone().requires_grad_() for t in _qkv(s=48))
    o = attention_reference(q, k, v, True, 1 / math.sqrt(q.shape[-1]))
    g = torch.Generator().manual_seed(9)
    o.backward(torch.randn(o.shape, generator=g))
    outs = run_distributed(_zigzag_worker, world)
    for i, ref in enumerate((o.detach(), q.grad, k.grad, v.grad)):
        got = unshard_sequence([out[i] for out in outs], "zigzag")
        assert torch.allclose(got, ref, atol=1e-5), (i, (got - ref).abs().max())


def _llama_zigzag_worker(rank, world):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.parallel.context_parallel import apply_context_parallel, shard_sequence

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=3)
    apply_context_parallel(m, dist.group.WORLD, "ring", layout="zigzag")
    g = torch.Generator().manual_seed(1)
    t = torch.randint(0, 128, (2, 33), generator=g)
    x = shard_sequence(t[:, :-1], dist.group.WORLD, "zigzag")
    y = shard_sequence(t[:, 1:], dist.group.WORLD, "zigzag")
    loss = m(x, y)
    loss.backward()
    gw = m.layers[0].attention.wqkv.weight.grad.clone()
    dist.all_reduce(gw)
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    return lt.item() / world, gw / world


def test_llama_zigzag_ring_matches_single():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=3)
    g = torch.Generator().manual_seed(1)
    t = torch.randint(0, 128, (2, 33), generator=g)
    loss = m(t[:, :-1], t[:, 1:])
    loss.backward()
    outs = run_distributed(_llama_zigzag_worker, 2)
    for lt, gw in outs:
        assert abs(lt - loss.item()) < 1e-5
        assert torch.allclose(gw, m.layers[0].attention.wqkv.weight.grad, atol=1e-5)


def _a2a_negative_dims_worker(rank, world):
    import torch

    from distributed_pytorch_hpc_amd.comm import functional as F

    torch.manual_seed(0)
    full = torch.randn(3, 4 * world, 6 * world, requires_grad=True)   # identical on every rank
    x = full.detach().chunk(world, 1)[rank].clone().requires_grad_()   # [3, 4, 6W]: sharded on dim 1
    out = {}
    for sd, gd in ((2, 1), (-1, -2), (-1, 1), (2, -2)):
        y = F.all_to_all(x, sd, gd, None)                              # -> [3, 4W, 6]: sharded on dim 2
        want = full.detach().chunk(world, 2)[rank]
        out[(sd, gd)] = bool(torch.equal(y, want))
        (g,) = torch.autograd.grad((y * y).sum(), x)
        out[(sd, gd, "grad")] = bool(torch.allclose(g, 2 * x.detach()))
    return out


def test_all_to_all_negative_dims():
    """all_to_all accepts negative scatter / gather dims (forward and backward) exactly like positive ones."""
    from dist_utils import run_distributed

    for res in run_distributed(_a2a_negative_dims_worker, 2):
        assert all(res.values()), res
