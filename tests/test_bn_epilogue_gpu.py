"""BatchNorm backward reduction in the consumer convolution's input-gradient epilogue (ops/conv.py BnGradSlot,
csrc/bn_epilogue.h, ``ts_gemm_nt_bnred``) against fp64 references of the same sums, and the ResNet blocks / ResNet-50
with the epilogue on vs off (DPH_BN_EPILOGUE=0: the BatchNorm's own reduction pass)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _kernels_on(monkeypatch):
    monkeypatch.setenv("DPH_CONV", "dph")
    monkeypatch.delenv("DPH_BN_EPILOGUE", raising=False)


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _mask(x, ss=None, bits=None):
    M, N = x.shape
    if bits is not None:
        return ((bits.long()[:, None] >> torch.arange(8, device=x.device)) & 1).reshape(M, N).bool()
    # the kernel's test is fmaf(x, scale, shift) > 0: in fp64 the product is exact and the sign of the sum survives
    return x.double() * ss[:N].double() + ss[N:].double() > 0


def _ref_sums(c, x, mean, invstd, mask):
    dz = c.double() * mask
    xh = (x.double() - mean.double()) * invstd.double()
    return dz.sum(0), (dz * xh).sum(0)


@pytest.mark.parametrize("form", ["1x1", "1x1_add", "1x1_sub", "3x3", "1x1_deep"])
@pytest.mark.parametrize("N", [64, 128, 256])
@pytest.mark.parametrize("mode", ["ss", "bits"])
def test_ts_gemm_nt_bnred_matches_fp64(dph_native, form, N, mode):
    """dX is bitwise the plain kernel's output; the partials sum to fp64 sum(dz) / sum(dz * xhat) over the stored bf16
    gradient, with a ragged last 128-row block."""
    torch.manual_seed(N + len(form))
    ops = torch.ops.dph
    n_img, H, W = 3, 9, 13                                  # M = 351: two full 128-row blocks + a ragged one
    M = n_img * H * W
    K = {"3x3": 64, "1x1_deep": 1024}.get(form, 128)   # deep K: the LDS-DMA one-tap GEMM (gemm1_lds_preferred)
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    if form == "3x3":
        b = (torch.randn(N, 9 * K, device=DEV) * 0.05).to(torch.bfloat16)
        ref = ops.ts_gemm_nt(a, b, H, W)
        hh, ww, add, sub = H, W, None, 0
    elif form == "1x1_sub":
        b = (torch.randn(N, K, device=DEV) * 0.1).to(torch.bfloat16)
        add = torch.randn(n_img * ((H + 1) // 2) * ((W + 1) // 2), N, device=DEV, dtype=torch.bfloat16)
        ref = ops.ts_gemm_nt_add_sub(a, b, add, H, W, 2)
        hh, ww, sub = H, W, 2
    else:
        b = (torch.randn(N, K, device=DEV) * 0.1).to(torch.bfloat16)
        add = torch.randn(M, N, device=DEV, dtype=torch.bfloat16) if form == "1x1_add" else None
        ref = ops.ts_gemm_nt(a, b, 0, 0, add)
        hh, ww, sub = 0, 0, 0
    x = (torch.randn(M, N, device=DEV) * 1.5 + 0.3).to(torch.bfloat16)
    mean = x.float().mean(0)
    invstd = torch.rsqrt(x.float().var(0, unbiased=False) + 1e-5)
    ss = bits = None
    if mode == "ss":
        ss = torch.cat([torch.randn(N, device=DEV), torch.randn(N, device=DEV) * 0.5])
    else:
        bits = torch.randint(0, 256, (M * N // 8,), device=DEV, dtype=torch.uint8)
    c, part = ops.ts_gemm_nt_bnred(a, b, hh, ww, add, sub, x, mean, invstd, ss, bits)
    torch.cuda.synchronize()
    assert torch.equal(c, ref)
    assert part.shape == ((M + 127) // 128, 2 * N)
    sd, sdx = _ref_sums(c, x, mean, invstd, _mask(x, ss, bits))
    got = part.double().sum(0)
    assert rel_err(got[:N], sd) < 1e-5
    assert rel_err(got[N:], sdx) < 1e-5


@pytest.mark.parametrize("residual", [False, True])
def test_bn_act_bwd_pre_part_matches_own_reduction(dph_native, residual):
    """bn_act_bwd with the epilogue's partials gives the dx / dgamma / dbeta of its own reduction pass (fp32 sums in
    another order: agreement to fp32 rounding)."""
    torch.manual_seed(3)
    ops = torch.ops.dph
    B, C, H, W = 4, 128, 10, 12
    x = torch.randn(B, C, H, W, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x) if residual else None
    w = (1 + 0.1 * torch.randn(C, device=DEV))
    bias = 0.1 * torch.randn(C, device=DEV)
    bits = torch.empty(x.numel() // 8, device=DEV, dtype=torch.uint8) if residual else None
    y, mean, invstd, ss = ops.bn_act_fwd(x, res, w, bias, None, None, 0.1, 1e-5, True, None, None, bits)
    A = torch.randn(B * H * W, 256, device=DEV, dtype=torch.bfloat16)
    Bw = (torch.randn(C, 256, device=DEV) * 0.05).to(torch.bfloat16)
    dy2, part = ops.ts_gemm_nt_bnred(A, Bw, 0, 0, None, 0, x, mean, invstd, None if residual else ss, bits)
    dy = dy2.view(B, H, W, C).permute(0, 3, 1, 2)
    saved = bits if residual else None
    kw = dict(xmask_ss=None if residual else ss, relu_mask=saved)
    ref = ops.bn_act_bwd(dy, x, x, mean, invstd, w, True, residual, True, **kw)
    got = ops.bn_act_bwd(dy, x, x, mean, invstd, w, True, residual, True, **kw, pre_part=part)
    for g_, r_ in zip(got, ref):
        if r_.numel():
            assert rel_err(g_, r_) < 1e-4


class _Count:
    def __init__(self, monkeypatch):
        from distributed_pytorch_hpc_amd.ops import conv as conv_mod

        self.used = 0
        orig = conv_mod.BnGradSlot.take

        def take(slot, dy):
            part = orig(slot, dy)
            self.used += part is not None
            return part

        monkeypatch.setattr(conv_mod.BnGradSlot, "take", take)


def _grads(model, x, monkeypatch, on):
    monkeypatch.setenv("DPH_BN_EPILOGUE", "1" if on else "0")
    model.zero_grad(set_to_none=True)
    x.grad = None
    torch.manual_seed(11)
    y = model(x)
    (y.float() * torch.randn_like(y.float())).sum().backward()
    torch.cuda.synchronize()
    return x.grad.double().clone(), {n: p.grad.double().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("kind", ["identity", "downsample", "basic"])
def test_blocks_epilogue_on_matches_off(dph_native, monkeypatch, kind):
    """A ResNet block pair (so the second block's conv1 reduces the first block's bn3): input and parameter gradients
    with the reductions in the convolution epilogues match the BatchNorms' own reduction passes."""
    import importlib

    R = importlib.import_module("distributed_pytorch_hpc_amd.models.resnet")
    torch.manual_seed(0)
    if kind == "identity":
        blocks = [R.Bottleneck(256, 64), R.Bottleneck(256, 64)]
        expect, cin, hw = 5, 256, 14   # bn1 x2 (3x3 consumer), bn2 x2 (conv3), first bn3 (second conv1)
    elif kind == "downsample":
        ds = torch.nn.Sequential(R.conv1x1(256, 512, 2), R.BatchNormAct2d(512, act=False))
        blocks = [R.Bottleneck(256, 64), R.Bottleneck(256, 128, 2, ds)]
        expect, cin, hw = 4, 256, 14   # bn1 (stride-1 block only), bn2 x2, first bn3 (conv1 + downsample slot)
    else:
        blocks = [R.BasicBlock(64, 64), R.BasicBlock(64, 64)]
        expect, cin, hw = 2, 64, 12    # bn1 x2 (conv2 consumers); bn2 outputs feed the next block's 3x3 conv1
    R.link_bn_handoff(blocks)
    model = torch.nn.Sequential(*blocks).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for m in model.modules():   # non-trivial affine parameters
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(4, cin, hw, hw, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    cnt = _Count(monkeypatch)
    gx0, g0 = _grads(model, x, monkeypatch, False)
    assert cnt.used == 0
    gx1, g1 = _grads(model, x, monkeypatch, True)
    assert cnt.used == expect
    assert rel_err(gx1, gx0) < 1e-2
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 1e-2, n


@pytest.mark.parametrize("hooks", [False, True])
def test_resnet50_epilogue_reductions_all_used(dph_native, monkeypatch, hooks):
    """ResNet-50 training step: 45 of the 53 BatchNorm backward reductions run in the consumers' gradient kernels (bn1
    of the 13 stride-1 conv2 blocks, every bn2, every bn3 but the last in convolution epilogues; the stem's in the
    max-pool gather), and the gradients match the unfused reductions.
    BatchNorm shifts at 3, as in tests/test_whole_net_grad_gpu.py: with the default init a random bf16 ResNet-50
    amplifies any change of fp32 summation order layer over layer (there: bf16 vs fp32 decorrelate completely).
    hooks: a full backward pre-hook on every block, as the FSDP engine installs (parallel/fsdp.py) -- the blocks then
    see aliases of each other's outputs, and the hand-off must still find them (models/resnet.py BnHandoff)."""
    from distributed_pytorch_hpc_amd.models.resnet import Bottleneck, resnet50

    torch.manual_seed(0)
    model = resnet50(num_classes=10, channels_last=True).to(DEV).to(torch.bfloat16)
    if hooks:
        for m in model.modules():
            if isinstance(m, Bottleneck):
                m.register_full_backward_pre_hook(lambda mod, g: None)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.bias.data.fill_(3.0)
    x = torch.randn(2, 3, 64, 64, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    cnt = _Count(monkeypatch)
    _, g0 = _grads(model, x, monkeypatch, False)
    _, g1 = _grads(model, x, monkeypatch, True)
    assert cnt.used == 45
    agg = rel_err(torch.cat([g1[n].flatten() for n in g0]), torch.cat([g0[n].flatten() for n in g0]))
    assert agg < 5e-3, agg
    for n in g0:
        if "conv" in n or "downsample.0" in n:
            assert rel_err(g1[n], g0[n]) < 5e-2, n


@pytest.mark.parametrize("N", [64, 256])
@pytest.mark.parametrize("reduce", [False, True])
def test_masked_residual_add_is_bitwise_the_materialised_add(dph_native, N, reduce):
    """ts_gemm_nt_addmask / ts_gemm_nt_bnred(add_mask=): A B^T + add * bits equals the plain add of the materialised
    bf16 masked gradient bit for bit (and the reduction partials match too)."""
    torch.manual_seed(N)
    ops = torch.ops.dph
    M, K = 333, 128
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = (torch.randn(N, K, device=DEV) * 0.1).to(torch.bfloat16)
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    bits = torch.randint(0, 256, (M * N // 8,), device=DEV, dtype=torch.uint8)
    dres = torch.where(_mask(dy, bits=bits), dy, torch.zeros_like(dy))
    ref = ops.ts_gemm_nt(a, b, 0, 0, dres)
    if not reduce:
        assert torch.equal(ops.ts_gemm_nt_addmask(a, b, dy, bits), ref)
        return
    x = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    mean, invstd = x.float().mean(0), torch.rsqrt(x.float().var(0, unbiased=False) + 1e-5)
    xbits = torch.randint(0, 256, (M * N // 8,), device=DEV, dtype=torch.uint8)
    c1, p1 = ops.ts_gemm_nt_bnred(a, b, 0, 0, dy, 0, x, mean, invstd, None, xbits, bits)
    c0, p0 = ops.ts_gemm_nt_bnred(a, b, 0, 0, dres, 0, x, mean, invstd, None, xbits)
    assert torch.equal(c1, ref) and torch.equal(c0, ref)
    assert torch.equal(p1, p0)


def test_identity_blocks_residual_mask_handoff_bitwise(dph_native, monkeypatch):
    """bn3 handing conv1 its dy + ReLU bits (DPH_RES_MASK=1, default) instead of the masked copy changes no bit of any
    gradient."""
    import importlib

    R = importlib.import_module("distributed_pytorch_hpc_amd.models.resnet")
    torch.manual_seed(0)
    blocks = [R.Bottleneck(256, 64), R.Bottleneck(256, 64), R.Bottleneck(256, 64)]
    R.link_bn_handoff(blocks)
    model = torch.nn.Sequential(*blocks).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("DPH_RES_MASK", v)
        out.append(_grads(model, x, monkeypatch, True))
    (gx0, g0), (gx1, g1) = out
    assert torch.equal(gx0, gx1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n


@pytest.mark.parametrize("stride", [1, 2])
def test_projection_shortcut_dual_bn_bitwise(dph_native, monkeypatch, stride):
    """bn3 + the downsample BatchNorm applied in one pass (ops.batchnorm.bn_dual_act, DPH_BN_DUAL=1 default) and
    their backward on dy + ReLU bits: output, every gradient, the running statistics and the batch counters are
    bitwise those of the two module calls (DPH_BN_DUAL=0)."""
    import copy
    import importlib

    R = importlib.import_module("distributed_pytorch_hpc_amd.models.resnet")
    torch.manual_seed(1)
    cout = 128 * 4
    ds = torch.nn.Sequential(R.conv1x1(256, cout, stride), R.BatchNormAct2d(cout, act=False))
    base = R.Bottleneck(256, 128, stride, ds).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for m in base.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x0 = torch.randn(4, 256, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for v in ("0", "1"):
        monkeypatch.setenv("DPH_BN_DUAL", v)
        blk = copy.deepcopy(base)
        x = x0.clone().requires_grad_()
        torch.manual_seed(5)
        y = blk(x)
        (y.float() * torch.randn_like(y.float())).sum().backward()
        torch.cuda.synchronize()
        bufs = {n: b.clone() for n, b in blk.named_buffers()}
        res.append((y.detach().clone(), x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters()}, bufs))
    (y0, gx0, g0, b0), (y1, gx1, g1, b1) = res
    assert torch.equal(y0, y1)
    assert torch.equal(gx0, gx1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    for n in b0:
        assert torch.equal(b0[n], b1[n]), n


@pytest.mark.parametrize("C", [64, 256])
def test_segment_merge_large_partial_counts(dph_native, C):
    """Thousands of per-tile partials are merged into segment rows before the finalize, in both directions
    (bn_merge_k / bn_bwd_merge_k): forward statistics / running stats / batch counter and backward dx / dgamma / dbeta
    match the BatchNorm's own passes, and repeated launches agree bit for bit."""
    torch.manual_seed(C)
    ops = torch.ops.dph
    B, H, W = 24, 100, 80                                    # M = 192 000 rows: 1 500 partials of 128 rows
    M = B * H * W
    a = torch.randn(M, 128, device=DEV, dtype=torch.bfloat16)
    wt = (torch.randn(C, 128, device=DEV) * 0.1 + 0.01).to(torch.bfloat16)
    y2, st = ops.ts_gemm_nt_stats(a, wt)
    x = y2.view(B, H, W, C).permute(0, 3, 1, 2)
    w = (1 + 0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    bias = (0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    outs = []
    for pre in (None, st, st):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        nbt = torch.zeros((), device=DEV, dtype=torch.long)
        r = ops.bn_act_fwd(x, None, w, bias, rm, rv, 0.1, 1e-5, True, pre, nbt)
        torch.cuda.synchronize()
        outs.append((r, rm, rv, nbt))
    (r0, rm0, rv0, n0), (r1, rm1, rv1, n1), (r2, rm2, rv2, n2) = outs
    for g_, ref in zip(r1, r0):
        assert rel_err(g_, ref) < 1e-4
    assert rel_err(rm1, rm0) < 1e-4 and rel_err(rv1, rv0) < 1e-4 and n1.item() == n0.item() == 1
    for g_, ref in zip(r2, r1):
        assert torch.equal(g_, ref)
    _, mean, invstd, ss = r1
    A = torch.randn(M, 256, device=DEV, dtype=torch.bfloat16)
    Bw = (torch.randn(C, 256, device=DEV) * 0.05).to(torch.bfloat16)
    dy2, part = ops.ts_gemm_nt_bnred(A, Bw, 0, 0, None, 0, x, mean, invstd, ss, None)
    dy = dy2.view(B, H, W, C).permute(0, 3, 1, 2)
    ref = ops.bn_act_bwd(dy, x, x, mean, invstd, w, True, False, True, ss)
    got = [ops.bn_act_bwd(dy, x, x, mean, invstd, w, True, False, True, ss, None, None, None, part) for _ in range(2)]
    torch.cuda.synchronize()
    for g_, r_ in zip(got[0], ref):
        if r_.numel():
            assert rel_err(g_, r_) < 1e-4
    for g_, r_ in zip(got[1], got[0]):
        assert torch.equal(g_, r_)


def test_stem_maxpool_gather_reduces_bn(dph_native, monkeypatch):
    """ResNet stem: the max-pool's gradient gather also runs the stem BatchNorm's backward reduction
    (maxpool_s2_bwd_bnred); dx is bitwise the plain gather and the partials sum to the fp64 reduction."""
    torch.manual_seed(2)
    ops = torch.ops.dph
    N, C, H, W = 4, 64, 30, 26
    x = (torch.randn(N, C, H, W, device=DEV) * 1.3 + 0.2).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y, mean, invstd, ss = ops.bn_act_fwd(x, None, None, None, None, None, 0.1, 1e-5, True)
    p, tap = ops.maxpool_s2_fwd(y, 3)
    dy = torch.randn_like(p)
    ref = ops.maxpool_s2_bwd(dy, tap, H, W, 3)
    dx, part = ops.maxpool_s2_bwd_bnred(dy, tap, H, W, 3, x, mean, invstd, ss)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
    sd, sdx = _ref_sums(dx.permute(0, 2, 3, 1).reshape(-1, C), x2, mean, invstd, _mask(x2, ss=ss))
    got = part.double().sum(0)
    assert rel_err(got[:C], sd) < 1e-5 and rel_err(got[C:], sdx) < 1e-5


def test_unet_conv_block_first_bn_reduced_in_second_conv(dph_native, monkeypatch):
    """SimpleUNet conv block: the first BatchNorm's backward reduction runs in the second 3x3 convolution's dgrad
    epilogue (biased conv path); gradients match the BatchNorm's own reduction."""
    from distributed_pytorch_hpc_amd.models.unet import conv_block

    torch.manual_seed(4)
    blk = conv_block(64, 128).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(2, 64, 24, 40, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    cnt = _Count(monkeypatch)
    gx0, g0 = _grads(blk, x, monkeypatch, False)
    assert cnt.used == 0
    gx1, g1 = _grads(blk, x, monkeypatch, True)
    assert cnt.used == 1
    assert rel_err(gx1, gx0) < 1e-2
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 1e-2, n


def test_simple_unet_all_bn_reductions_in_consumers(dph_native, monkeypatch):
    """Whole SimpleUNet: every block's first BatchNorm reduces in its second convolution (7), the bottleneck /
    decoder blocks' last BatchNorm in the up-path GEMM or the output 1x1 convolution (4), and the encoder blocks' last
    BatchNorm in the max pooling's gather, which also adds the skip gradient (3); gradients match the BatchNorms' own
    reduction passes."""
    from distributed_pytorch_hpc_amd.models.unet import SimpleUNet, to_channels_last

    torch.manual_seed(5)
    net = to_channels_last(SimpleUNet(65, 65, 64).to(DEV).to(torch.bfloat16))
    x = torch.randn(2, 65, 48, 80, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    cnt = _Count(monkeypatch)
    gx0, g0 = _grads(net, x, monkeypatch, False)
    assert cnt.used == 0
    gx1, g1 = _grads(net, x, monkeypatch, True)
    assert cnt.used == 14
    assert rel_err(gx1, gx0) < 2e-2
    num = sum((g1[n] - g0[n]).norm() ** 2 for n in g0) ** 0.5
    den = sum(g0[n].norm() ** 2 for n in g0) ** 0.5
    assert num / den < 1e-2


def test_simple_unet_skip_gradient_in_pool_is_bitwise(dph_native, monkeypatch):
    """The skip connection's gradient added in the max pooling's gather (ops.pool.SkipGradSlot) instead of autograd's
    add: with the BatchNorms' own reductions (DPH_BN_EPILOGUE=0) the input and parameter gradients are bitwise the
    same as with the copy + add."""
    from distributed_pytorch_hpc_amd.models.unet import SimpleUNet, to_channels_last

    torch.manual_seed(6)
    net = to_channels_last(SimpleUNet(65, 65, 64).to(DEV).to(torch.bfloat16))
    x = torch.randn(2, 65, 45, 90, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    monkeypatch.setenv("DPH_UNET_SKIP_FOLD", "0")
    gx0, g0 = _grads(net, x, monkeypatch, False)
    monkeypatch.setenv("DPH_UNET_SKIP_FOLD", "1")
    gx1, g1 = _grads(net, x, monkeypatch, False)
    assert torch.equal(gx1, gx0)
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("k,C,H,W", [(2, 64, 45, 90), (2, 256, 12, 23), (3, 64, 28, 28)])
def test_maxpool_bwd_add_operand(dph_native, k, C, H, W):
    """maxpool_s2_bwd / maxpool_s2_bwd_bnred with a second gradient read from a channel slice of a wider tensor:
    bitwise the bf16 sum of the plain gather and the slice; the BatchNorm partials match a float64 reduction of it."""
    torch.manual_seed(C + H)
    ops = torch.ops.dph
    N, off = 2, 32
    x = torch.randn(N, C, H, W, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    _, tap = ops.maxpool_s2_fwd(x, k)
    ho, wo = (H - 1) // 2 + 1 if k == 3 else H // 2, (W - 1) // 2 + 1 if k == 3 else W // 2
    dy = torch.randn(N, C, ho, wo, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wide = torch.randn(N, off + C + 16, H, W, device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    sl = wide[:, off:off + C]
    ref = ops.maxpool_s2_bwd(dy, tap, H, W, k) + sl
    got = ops.maxpool_s2_bwd(dy, tap, H, W, k, wide, off)
    assert torch.equal(got, ref)
    mean = torch.randn(C, device=DEV) * 0.1
    invstd = torch.rand(C, device=DEV) + 0.5
    ss = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1])
    dx, part = ops.maxpool_s2_bwd_bnred(dy, tap, H, W, k, x, mean, invstd, ss, wide, off)
    assert torch.equal(dx, ref)
    xf = x.double().permute(0, 2, 3, 1).reshape(-1, C)
    on = (xf * ss[:C].double() + ss[C:].double()) > 0
    dz = torch.where(on, dx.double().permute(0, 2, 3, 1).reshape(-1, C), torch.zeros((), device=DEV,
                                                                                    dtype=torch.float64))
    xhat = (xf - mean.double()) * invstd.double()
    p = part.double().sum(0)
    assert rel_err(p[:C], dz.sum(0)) < 1e-4
    assert rel_err(p[C:], (dz * xhat).sum(0)) < 1e-4


@pytest.mark.parametrize("M,K,N", [(50176 // 8, 1024, 256), (12544 // 4 + 37, 2048, 512), (777, 1024, 128)])
def test_deep_1x1_on_lds_dma_gemm(dph_native, M, K, N):
    """Deep-K 1x1 GEMMs (K >= 1024) run on the LDS-DMA implicit GEMM with a one-tap identity geometry: the product
    matches fp32, and the BatchNorm-statistics epilogue drives bn_act_fwd like its own statistics pass."""
    torch.manual_seed(K + N)
    ops = torch.ops.dph
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = (torch.randn(N, K, device=DEV) * 0.03).to(torch.bfloat16)
    y = ops.ts_gemm_nt(a, b)
    ref = a.float() @ b.float().t()
    assert rel_err(y, ref) < 1e-2
    y2, st = ops.ts_gemm_nt_stats(a, b)
    assert torch.equal(y2, y)
    x = y2.view(1, M, 1, N).permute(0, 3, 1, 2)   # channels-last [1, N, M, 1] view of the [M, N] rows
    r0 = ops.bn_act_fwd(x, None, None, None, None, None, 0.1, 1e-5, True)
    r1 = ops.bn_act_fwd(x, None, None, None, None, None, 0.1, 1e-5, True, st)
    for g_, r_ in zip(r1, r0):
        assert rel_err(g_, r_) < 1e-4


def test_dual_bn_fused_dx_pass_matches_two_passes(dph_native, monkeypatch):
    """The projection shortcut's backward with both BatchNorms' dx in one pass (bn_bwd_dx2_k, DPH_BN_DUAL_DX=1
    default) gives the same gradients as two single passes."""
    import copy
    import importlib

    R = importlib.import_module("distributed_pytorch_hpc_amd.models.resnet")
    torch.manual_seed(3)
    ds = torch.nn.Sequential(R.conv1x1(256, 512, 2), R.BatchNormAct2d(512, act=False))
    base = R.Bottleneck(256, 128, 2, ds).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for m in base.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x0 = torch.randn(4, 256, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for v in ("0", "1"):
        monkeypatch.setenv("DPH_BN_DUAL_DX", v)
        blk = copy.deepcopy(base)
        x = x0.clone().requires_grad_()
        torch.manual_seed(5)
        y = blk(x)
        (y.float() * torch.randn_like(y.float())).sum().backward()
        torch.cuda.synchronize()
        res.append((x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters()}))
    (gx0, g0), (gx1, g1) = res
    assert rel_err(gx1, gx0) < 1e-5
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 1e-5, n
