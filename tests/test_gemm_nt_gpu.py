"""Numerics of the CDNA4 forward / input-gradient GEMM (csrc/gemm_nt.hip) and its fused epilogues against plain
PyTorch fp32 references of the same ops (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (scale * torch.randn(*shape, device=DEV, generator=g)).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (768, 512, 320), (256, 1024, 4096),
                                   (2048, 256, 128)])
def test_gemm_nt_store(dph_native, M, N, K):
    a, b = _rnd(M, K, seed=1), _rnd(N, K, seed=2)
    c = dph_native.gemm_nt(a, b)
    ref = a.float() @ b.float().t()
    assert c.shape == (M, N) and c.dtype == torch.bfloat16
    assert rel_err(c, ref) < 5e-3
    # every output element is written (no tile left unvisited): worst element within bf16 rounding of the ref
    assert ((c.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-2 * ref.abs().mean()).all()


def test_gemm_nt_store_asymmetric_identity(dph_native):
    """A = I with an asymmetric B: a transposed store or a swapped row / column map shows up exactly."""
    M = N = K = 256
    a = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(N * K, device=DEV) % 251).reshape(N, K).to(torch.bfloat16)
    c = dph_native.gemm_nt(a, b)
    assert torch.equal(c, b.t().contiguous())


def test_gemm_nt_3d_input(dph_native):
    a, b = _rnd(2, 256, 128, seed=3), _rnd(512, 128, seed=4)
    c = dph_native.gemm_nt(a, b)
    assert c.shape == (2, 256, 512)
    assert rel_err(c, a.float() @ b.float().t()) < 5e-3


@pytest.mark.parametrize("M,H,K", [(256, 128, 64), (512, 384, 256), (256, 11008 // 8 * 8 // 128 * 128, 512)])
def test_gemm_nt_swiglu(dph_native, M, H, K):
    x, w13 = _rnd(M, K, seed=5), _rnd(2 * H, K, seed=6, scale=0.5)
    x13, h = dph_native.gemm_nt_swiglu(x, w13)
    ref13 = x.float() @ w13.float().t()
    assert x13.shape == (M, 2 * H) and h.shape == (M, H)
    assert rel_err(x13, ref13) < 5e-3
    g, u = ref13[:, :H], ref13[:, H:]
    assert rel_err(h, torch.nn.functional.silu(g) * u) < 1e-2
    # h is exactly the separate SwiGLU kernel applied to the fused kernel's own (rounded) gate / up
    assert torch.equal(h, dph_native.swiglu_fwd(x13))


@pytest.mark.parametrize("M,H,K", [(256, 256, 64), (512, 512, 256), (768, 768, 128)])
def test_gemm_nt_dswiglu(dph_native, M, H, K):
    dy, w2t = _rnd(M, K, seed=7), _rnd(H, K, seed=8, scale=0.5)
    x13 = _rnd(M, 2 * H, seed=9, scale=2.0)
    d13 = dph_native.gemm_nt_dswiglu(dy, w2t, x13)
    dh = dy.float() @ w2t.float().t()
    g, u = x13[:, :H].float(), x13[:, H:].float()
    s = torch.sigmoid(g)
    ref = torch.cat([dh * u * s * (1 + g * (1 - s)), dh * g * s], 1)
    assert d13.shape == (M, 2 * H)
    assert rel_err(d13, ref) < 1e-2
    # the epilogue is the separate SwiGLU backward applied to the kernel's rounded dh
    dh_k = dph_native.gemm_nt(dy, w2t)
    assert rel_err(d13, dph_native.swiglu_bwd(dh_k, x13)) < 2e-3


@pytest.mark.parametrize("S,hd,heads", [(256, 64, 4), (512, 128, 2)])
def test_gemm_nt_rope(dph_native, S, hd, heads):
    from distributed_pytorch_hpc_amd.models.llama2 import rope_tables

    B, K = 2, 256
    N = 3 * heads * hd                        # q | k | v
    x, w = _rnd(B * S, K, seed=10), _rnd(N, K, seed=11, scale=0.2)
    cos, sin = rope_tables(hd, 2 * S, 10000.0, torch.device(DEV))
    for pos_off in (0, 7):
        y = dph_native.gemm_nt_rope(x, w, cos, sin, S, hd, 2 * heads * hd, pos_off)
        ref = x.float() @ w.float().t()
        pos = torch.arange(B * S, device=DEV) % S + pos_off
        c, s = cos[pos], sin[pos]                                         # [rows, hd/2]
        rot = ref[:, :2 * heads * hd].reshape(B * S, 2 * heads, hd // 2, 2)
        a, b = rot[..., 0], rot[..., 1]
        c, s = c[:, None, :], s[:, None, :]
        rot = torch.stack([a * c - b * s, a * s + b * c], -1).reshape(B * S, -1)
        ref = torch.cat([rot, ref[:, 2 * heads * hd:]], 1)
        assert rel_err(y, ref) < 5e-3, pos_off


def _tiny_llama(seed):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    # dim 256, FFN 768, 2 heads of 128: every projection tiles the NT kernel (rows 2 x 256, N % 256, K % 64)
    args = ModelArgs(dim=256, n_layers=2, n_heads=2, vocab_size=512, multiple_of=256, max_seq_len=512)
    return build_llama(args, device=DEV, dtype=torch.bfloat16, seed=seed)


@pytest.mark.parametrize("which", ["mlp", "mlp_bwd", "qkv", "both"])
def test_llama_fused_blocks_match_unfused(dph_native, which):
    """Loss and every parameter gradient of a Llama with the fused SwiGLU-MLP / QKV+RoPE+attention paths against
    the same model through the unfused modules (library GEMMs + separate SwiGLU / RoPE kernels)."""
    from distributed_pytorch_hpc_amd.parallel import fused_layers

    g = torch.Generator(device=DEV).manual_seed(0)
    t = torch.randint(0, 512, (2, 257), device=DEV, generator=g)
    out = {}
    for fused in (False, True):
        mlp = ("bwd" if which == "mlp_bwd" else True) if fused and which != "qkv" else False
        old = fused_layers.set_enabled(mlp=mlp, qkv=fused and which in ("qkv", "both"))
        try:
            m = _tiny_llama(3)
            ff = m.layers[0].feed_forward
            at = m.layers[0].attention
            x = torch.randn(2, 256, 256, device=DEV, dtype=torch.bfloat16)
            if fused and which != "qkv":
                assert fused_layers.swiglu_mlp_ok(x, ff.w13, ff.w2)
            if fused and which in ("qkv", "both"):
                assert fused_layers.qkv_rope_attention_ok(x, at.wqkv, at.head_dim)
            loss = m(t[:, :-1], t[:, 1:])
            loss.backward()
            out[fused] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()})
        finally:
            fused_layers.set_enabled(*old)
    (l0, g0), (l1, g1) = out[False], out[True]
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 3e-2, n


def _check_store(c, ref):
    assert rel_err(c, ref) < 5e-3
    assert ((c.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-2 * ref.abs().mean()).all()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (768, 512, 320), (256, 1024, 4096),
                                   # ragged: tp8 / tp4 shards of Llama-2-7B (w13 2752, head 4000, w2's K 1376),
                                   # a partial single K-tile, the smallest N
                                   (256, 2752, 256), (512, 4000, 128), (256, 4096, 1376), (256, 520, 40),
                                   (256, 8, 72), (512, 1000, 200)])
def test_gemm_nt_ragged_store(dph_native, M, N, K):
    a, b = _rnd(M, K, seed=21), _rnd(N, K, seed=22)
    c = (dph_native.gemm_nt(a, b))
    assert c.shape == (M, N)
    _check_store(c, a.float() @ b.float().t())


def test_gemm_nt_ragged_asymmetric_identity(dph_native):
    M = N = K = 256
    a = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(N * K, device=DEV) % 251).reshape(N, K).to(torch.bfloat16)
    c = (dph_native.gemm_nt(a, b))
    assert torch.equal(c, b.t().contiguous())


@pytest.mark.parametrize("M,H,K", [(256, 128, 64), (512, 384, 256), (256, 1376, 256), (256, 2752, 136),
                                   (256, 40, 64)])
def test_gemm_nt_ragged_swiglu(dph_native, M, H, K):
    x, w13 = _rnd(M, K, seed=25), _rnd(2 * H, K, seed=26, scale=0.5)
    x13, h = (dph_native.gemm_nt_swiglu(x, w13))
    ref13 = x.float() @ w13.float().t()
    assert x13.shape == (M, 2 * H) and h.shape == (M, H)
    assert rel_err(x13, ref13) < 5e-3
    g, u = ref13[:, :H], ref13[:, H:]
    assert rel_err(h, torch.nn.functional.silu(g) * u) < 1e-2
    assert torch.equal(h, dph_native.swiglu_fwd(x13))


@pytest.mark.parametrize("M,H,K", [(256, 256, 64), (512, 768, 128), (256, 1376, 512), (256, 2752, 200)])
def test_gemm_nt_ragged_dswiglu(dph_native, M, H, K):
    dy, w2t = _rnd(M, K, seed=27), _rnd(H, K, seed=28, scale=0.5)
    x13 = _rnd(M, 2 * H, seed=29, scale=2.0)
    d13 = (dph_native.gemm_nt_dswiglu(dy, w2t, x13))
    dh = dy.float() @ w2t.float().t()
    g, u = x13[:, :H].float(), x13[:, H:].float()
    s = torch.sigmoid(g)
    ref = torch.cat([dh * u * s * (1 + g * (1 - s)), dh * g * s], 1)
    assert d13.shape == (M, 2 * H)
    assert rel_err(d13, ref) < 1e-2


@pytest.mark.parametrize("S,hd,heads,K", [(256, 64, 4, 256), (512, 128, 2, 256), (256, 128, 4, 1376)])
def test_gemm_nt_ragged_rope(dph_native, S, hd, heads, K):
    from distributed_pytorch_hpc_amd.models.llama2 import rope_tables

    B = 2
    N = 3 * heads * hd
    x, w = _rnd(B * S, K, seed=30), _rnd(N, K, seed=31, scale=0.2)
    cos, sin = rope_tables(hd, 2 * S, 10000.0, torch.device(DEV))
    y = dph_native.gemm_nt_rope(x, w, cos, sin, S, hd, 2 * heads * hd, 3)
    ref = x.float() @ w.float().t()
    pos = torch.arange(B * S, device=DEV) % S + 3
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    rot = ref[:, :2 * heads * hd].reshape(B * S, 2 * heads, hd // 2, 2)
    a, b = rot[..., 0], rot[..., 1]
    rot = torch.stack([a * c - b * s, a * s + b * c], -1).reshape(B * S, -1)
    assert rel_err(y, torch.cat([rot, ref[:, 2 * heads * hd:]], 1)) < 5e-3

@pytest.mark.parametrize("variant", [4, 5, 6, 7])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (768, 512, 320), (256, 1024, 4096),
                                   (2048, 256, 128), (1024, 512, 64 * 7)])
def test_gemm_nt4_store(dph_native, variant, M, N, K):
    """The 4-wave / 256-AGPR plain GEMM (gemm_nt4_k, every PIPE form): against the fp32 reference, bitwise equal to
    the 8-wave kernel, odd and even K-tile counts, and the identity check for the row / column map."""
    a, b = _rnd(M, K, seed=1), _rnd(N, K, seed=2)
    ref8 = dph_native.gemm_nt(a, b)
    old = dph_native.gemm_nt_variant(variant)
    try:
        c = dph_native.gemm_nt(a, b)
        eye = torch.eye(256, 256, device=DEV, dtype=torch.bfloat16)
        asym = (torch.arange(256 * 256, device=DEV) % 251).reshape(256, 256).to(torch.bfloat16)
        ci = dph_native.gemm_nt(eye, asym)
    finally:
        dph_native.gemm_nt_variant(old)
    ref = a.float() @ b.float().t()
    assert rel_err(c, ref) < 5e-3
    assert ((c.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-2 * ref.abs().mean()).all()
    assert torch.equal(c, ref8)
    assert torch.equal(ci, asym.t().contiguous())
