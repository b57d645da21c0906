"""Serving kernels on the MI355X (csrc/decode.hip) against fp32 PyTorch references, and the HIP-graph decode loop."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _qkv(b, s, hq, hkv, d, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(b, s, (hq + 2 * hkv) * d, device="cuda", generator=g).to(torch.bfloat16)


@pytest.mark.parametrize("s", [1, 5])
def test_kv_append_fp8_cache_bitwise(dph_native, s):
    """The kernel's e4m3 entries equal torch's cast of the bf16 rotated key / value divided by the scale."""
    from distributed_pytorch_hpc_amd.ops.decode import kv_append_, kv_append_reference
    from distributed_pytorch_hpc_amd.ops.rope import precompute_rope_tables

    b, hq, hkv, d, smax = 3, 8, 2, 128, 64
    cos, sin = precompute_rope_tables(d, 128, device="cuda")
    pos = torch.tensor([0, 7, 20], dtype=torch.int32, device="cuda")
    qkv = _qkv(b, s, hq, hkv, d) * 40   # values past the e4m3 range saturate
    kc = torch.zeros(b, smax, hkv, d, dtype=torch.float8_e4m3fn, device="cuda")
    vc = torch.zeros_like(kc)
    q2, k2, v2 = qkv.clone(), kc.clone(), vc.clone()
    kv_append_(qkv, kc, vc, pos, cos, sin, hq, hkv, 0.5)
    # the reference rounds the rotated key through bf16 exactly as the kernel does
    kv_append_reference(q2, k2, v2, pos, cos, sin, hq, hkv, 0.5)
    assert torch.equal(vc.view(torch.uint8), v2.view(torch.uint8))
    diff = (kc.float() - k2.float()).abs()
    assert (diff > 0).float().mean() < 0.01   # rotation rounding (fma vs mul+add) may move a few values one step


@pytest.mark.parametrize("s", [1, 5])
def test_kv_append_matches_reference(dph_native, s):
    from distributed_pytorch_hpc_amd.ops.decode import kv_append_, kv_append_reference
    from distributed_pytorch_hpc_amd.ops.rope import precompute_rope_tables

    b, hq, hkv, d, smax = 3, 8, 2, 128, 64
    cos, sin = precompute_rope_tables(d, 128, device="cuda")
    pos = torch.tensor([0, 7, 20], dtype=torch.int32, device="cuda")
    qkv = _qkv(b, s, hq, hkv, d)
    kc = torch.zeros(b, smax, hkv, d, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros_like(kc)
    q2, k2, v2 = qkv.clone(), kc.clone(), vc.clone()
    kv_append_(qkv, kc, vc, pos, cos, sin, hq, hkv)
    kv_append_reference(q2, k2, v2, pos, cos, sin, hq, hkv)
    torch.testing.assert_close(qkv.float(), q2.float(), atol=1e-2, rtol=8e-3)   # one bf16 rounding apart at most
    torch.testing.assert_close(kc.float(), k2.float(), atol=1e-2, rtol=8e-3)
    assert torch.equal(vc, v2)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("hq,hkv,d", [(32, 32, 128), (8, 2, 128), (12, 4, 64), (16, 4, 32), (8, 1, 128)])
def test_decode_attention_matches_fp32_reference(dph_native, hq, hkv, d, fp8):
    from distributed_pytorch_hpc_amd.ops.decode import decode_attention, decode_attention_reference, quantize_kv

    b, smax, ks = 3, 300, 0.25
    pos = torch.tensor([0, 130, 299], dtype=torch.int32, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    kc = torch.randn(b, smax, hkv, d, device="cuda", generator=g).to(torch.bfloat16)
    vc = torch.randn(b, smax, hkv, d, device="cuda", generator=g).to(torch.bfloat16)
    for i, p in enumerate(pos.tolist()):   # past each sequence's end: NaN, which must never be read into o
        kc[i, p + 1:] = float("nan")
        vc[i, p + 1:] = float("nan")
    if fp8:   # e4m3 entries (NaN stays NaN through the cast)
        kc, vc = quantize_kv(kc, ks), quantize_kv(vc, ks)
    sc = ks if fp8 else 1.0
    qkv = _qkv(b, 1, hq, hkv, d, seed=2)
    ref = decode_attention_reference(qkv, kc, vc, pos, hq, hkv, 1.0 / math.sqrt(d), kv_scale=sc).float()
    for bound in (None, 300):   # launch over the capacity (graph mode) or a tight bound: same result
        out = decode_attention(qkv, kc, vc, pos, hq, hkv, max_len=bound, kv_scale=sc)
        assert out.shape == (b, hq * d) and torch.isfinite(out).all()
        torch.testing.assert_close(out.float(), ref, atol=1e-2, rtol=1e-2)


def _tiny_llama(seed=0):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    args = ModelArgs(dim=512, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=512, multiple_of=64, max_seq_len=256)
    return build_llama(args, device="cuda", dtype=torch.bfloat16, seed=seed)


def test_llama_serving_matches_full_forward_bf16(dph_native):
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _tiny_llama()
    t = torch.randint(0, 512, (2, 96), device="cuda", generator=torch.Generator(device="cuda").manual_seed(0))
    with torch.no_grad():
        full = m(t)
    c = KVCache(m, 2, 128)
    got = [m.forward_inference(t[:, :64], c)]
    for i in range(64, 96):
        got.append(m.forward_inference(t[:, i:i + 1], c))
    got = torch.stack(got, 1)
    ref = full[:, 63:96]
    rel = (got - ref).norm() / ref.norm()
    assert rel < 2e-2, rel
    assert (got.argmax(-1) == ref.argmax(-1)).float().mean() > 0.9


def test_generator_graph_replay_matches_eager(dph_native):
    from distributed_pytorch_hpc_amd.inference import Generator

    m = _tiny_llama(seed=3)
    prompts = [[5, 6, 7, 8, 9, 10], [11, 12, 13]]   # ragged: per-slot prefill, then batched decode
    eager = Generator(m, 2, 64, graphs=False).generate(prompts, 24)
    g = Generator(m, 2, 64, graphs=True)
    graphed = g.generate(prompts, 24)
    assert g._graph is not None
    assert graphed == eager
    assert g.generate(prompts, 24) == eager          # the captured graph is reused after reset


@pytest.mark.parametrize("m", [1, 2, 5, 16, 17, 40, 64])
@pytest.mark.parametrize("n,k", [(4096, 4096), (272, 11008), (96, 256), (40, 1000)])
def test_skinny_linear_matches_fp32(dph_native, m, n, k):
    from distributed_pytorch_hpc_amd.ops.decode import skinny_linear

    if (n % 16 or k % 128) and m > 2:
        pytest.skip("shape covered by the GEMV form only (1-2 rows)")
    g = torch.Generator(device="cuda").manual_seed(m + n)
    x = torch.randn(m, k, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).to(torch.bfloat16)
    y = skinny_linear(x, w)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    # strided rows (a view into a wider buffer) and a leading batch shape
    xb = torch.randn(m, 1, k + 256, device="cuda", generator=g).to(torch.bfloat16)[..., :k]
    torch.testing.assert_close(skinny_linear(xb, w).float(), (xb.float() @ w.float().t()), atol=2e-2, rtol=2e-2)


def test_producer_fused_gemv_matches_composition(dph_native):
    """RMSNorm(x + res) and SwiGLU computed inside the GEMV equal the separate kernels followed by the projection."""
    from distributed_pytorch_hpc_amd import ops
    from distributed_pytorch_hpc_amd.ops.decode import gemv_rmsnorm, gemv_swiglu, skinny_linear

    g = torch.Generator(device="cuda").manual_seed(7)
    k, n = 4096, 1024
    x = torch.randn(1, 1, k, device="cuda", generator=g).to(torch.bfloat16)
    res = torch.randn(1, 1, k, device="cuda", generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(k, device="cuda", generator=g)).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).to(torch.bfloat16)
    y, h = gemv_rmsnorm(x, res, nw, 1e-5, w)
    h_ref, a_ref = ops.add_rms_norm(x, res, nw, 1e-5)
    assert torch.equal(h, h_ref)
    torch.testing.assert_close(y.float(), skinny_linear(a_ref, w).float(), atol=2e-2, rtol=2e-2)
    y0, h0 = gemv_rmsnorm(x, None, nw, 1e-5, w)
    assert h0 is x
    torch.testing.assert_close(y0.float(), skinny_linear(ops.rms_norm(x, nw, 1e-5), w).float(), atol=2e-2, rtol=2e-2)
    for m in (1, 2):
        x2 = torch.randn(m, 1, 2 * 11008, device="cuda", generator=g).to(torch.bfloat16)
        w2 = (torch.randn(4096, 11008, device="cuda", generator=g) / 11008 ** 0.5).to(torch.bfloat16)
        torch.testing.assert_close(gemv_swiglu(x2, w2).float(), skinny_linear(ops.swiglu(x2), w2).float(), atol=2e-2,
                                   rtol=2e-2)


def test_batch1_fused_decode_matches_unfused(dph_native, monkeypatch):
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache
    from distributed_pytorch_hpc_amd.ops import decode as decode_ops

    m = _tiny_llama(seed=5)
    t = torch.randint(0, 512, (1, 40), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))

    def run():
        c = KVCache(m, 1, 64)
        out = [m.forward_inference(t[:, :32], c)]
        for i in range(32, 40):
            out.append(m.forward_inference(t[:, i:i + 1], c))
        return torch.stack(out, 1)

    fused = run()
    monkeypatch.setattr(decode_ops, "fused_decode_ok", lambda *a, **k: False)
    plain = run()
    assert (fused - plain).norm() / plain.norm() < 1e-2
    assert torch.equal(fused.argmax(-1), plain.argmax(-1))


def test_continuous_batching_graphs_match_eager(dph_native):
    from distributed_pytorch_hpc_amd.inference import ContinuousBatcher, Generator

    m = _tiny_llama(seed=9)
    reqs = [([5, 6, 7], 9), ([8, 9, 10, 11, 12, 13, 14], 4), ([15], 12), ([16, 17], 2), ([18, 19, 20, 21], 7)]

    def serve(graphs):
        cb = ContinuousBatcher(Generator(m, 2, 32, graphs=graphs))
        hs = [cb.submit(p, n) for p, n in reqs]
        cb.run()
        return [h.output for h in hs], cb.gen._graph is not None

    eager, _ = serve(False)
    graphed, captured = serve(True)
    assert captured and graphed == eager
    assert [len(o) for o in eager] == [n for _, n in reqs]


def test_llama_serving_fp8_kv_cache(dph_native):
    from distributed_pytorch_hpc_amd.inference import Generator
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _tiny_llama(seed=11)
    t = torch.randint(0, 512, (2, 72), device="cuda", generator=torch.Generator(device="cuda").manual_seed(4))

    def run(dtype):
        c = KVCache(m, 2, 128, dtype=dtype)
        out = [m.forward_inference(t[:, :64], c)]
        out += [m.forward_inference(t[:, i:i + 1], c) for i in range(64, 72)]
        return torch.stack(out, 1)

    bf, f8 = run(None), run(torch.float8_e4m3fn)
    assert (f8 - bf).norm() / bf.norm() < 0.05
    eager = Generator(m, 2, 64, graphs=False, dtype=torch.float8_e4m3fn).generate([[1, 2, 3], [4, 5, 6, 7]], 12)
    graphed = Generator(m, 2, 64, graphs=True, dtype=torch.float8_e4m3fn).generate([[1, 2, 3], [4, 5, 6, 7]], 12)
    assert graphed == eager
