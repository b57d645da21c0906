"""Whole-network bf16 gradient checks for the convolution models (GPU only).

The per-op tests pin each kernel against fp32; these pin the COMPOSED step the benches time: ResNet-50 under the
world-1 FSDP engine (bf16 parameters / activations / gradients, channels-last: stem, strided, 1x1 / 3x3 forward and
``c3w_k`` weight-gradient kernels, fused BatchNorm, the residual-gradient hand-offs) and SimpleUNet under the DDP
engine (65-channel edge convs, biased 3x3 convs with the BN-statistics epilogue, fused up-sample + concat, pooling,
latitude-weighted MSE).  Every parameter's gradient is compared with an fp32 ATen run of the same (bf16-representable)
weights and input, and with the bf16 ATen / MIOpen run of the same network as the yardstick of what bf16 alone costs.

Conditioning (benchmarks/probes/wholenet_conditioning.py, profiles/r5/wholenet/): a random-init BatchNorm-ReLU network
in training mode amplifies rounding layer over layer.  With the default BN init (shift 0, half the ReLU inputs
clipped) bf16 gradients of ResNet-50 are DECORRELATED from fp32 -- aggregate rel L2 1.30, min cosine -0.05 -- for
stock bf16 MIOpen exactly as for the framework (1.30 / 1.30), and SimpleUNet's land 0.13 / 0.14 away; no bf16
implementation can meet a fp32 bound there.  Every BatchNorm's shift is therefore set to 3 (the ReLUs clip ~0.1 %),
which keeps all kernels on their normal paths but stops the amplification: aggregate 0.0011 (ResNet-50) and 0.0021
(SimpleUNet).  Then:
  * loss within 2e-3 of fp32; whole-gradient rel L2 < 1e-2 and within 1.25x (+1e-3) of stock bf16's;
  * every parameter's error within noise of stock bf16's (1.25x + 2e-2; 1.5x + 5e-2 where stock bf16 is itself
    > 0.1 off, mostly BatchNorm shifts whose true gradient nearly cancels); a structurally-zero gradient (a conv
    bias under a BN) no larger than 3x stock bf16's noise;
  * every conv / linear weight gradient at cosine > 0.995 against fp32 (ResNet's stem: 0.985 -- its 3x3 max-pool
    routes gradients by bf16 ties, stock bf16 lands at 0.990 too);
  * SimpleUNet additionally: every parameter within rel 5e-2 and cosine 0.995 of fp32.
ResNet-50's per-parameter errors stay at 0.04-0.08 (weights) even so -- for stock bf16 MIOpen exactly as for the
framework (the bound is comparative there); SimpleUNet's are <= 0.02.
Reference: scripts/main.py:308-339 (ResNet training loop), scripts/01_data_parallel_ddp/multinode_ddp_unet.py:174-192.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _stats(got: torch.Tensor, ref: torch.Tensor):
    g, r = got.float().flatten(), ref.float().flatten()
    rel = ((g - r).norm() / r.norm().clamp_min(1e-20)).item()
    cos = F.cosine_similarity(g, r, dim=0).item() if r.norm() > 0 else 1.0
    return rel, cos


def _grads_reference(model32, x, loss_fn, dtype):
    """Gradients of an ATen-only run (the stock-op comparator mode) in ``dtype``."""
    from distributed_pytorch_hpc_amd.ops import _lib

    m = copy.deepcopy(model32).to(dtype)
    _lib.set_reference_mode(True)
    try:
        loss = loss_fn(m(x.to(dtype)))
        loss.backward()
    finally:
        _lib.set_reference_mode(False)
    return loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def _rows(model32, x, loss_fn, wrap):
    """Per-parameter (name, rel, cos, rel_aten_bf16, cos_aten_bf16, |g32|, |g|, |g_aten_bf16|) of the framework's
    bf16 gradients and of stock ATen bf16's, each against the fp32 ATen run; plus the three losses."""
    from distributed_pytorch_hpc_amd.parallel.data_parallel import MixedPrecision

    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        l32, g32 = _grads_reference(model32, x, loss_fn, torch.float32)
        lbf, gbf = _grads_reference(model32, x, loss_fn, torch.bfloat16)
    finally:
        torch.backends.cudnn.deterministic = det
    model = copy.deepcopy(model32)
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16)
    wrapped = wrap(model, mp)
    loss = loss_fn(wrapped(x.to(torch.bfloat16)))
    loss.backward()
    wrapped.synchronize() if hasattr(wrapped, "synchronize") else wrapped.engine.synchronize()
    torch.cuda.synchronize()
    rows = []
    for n, p in model.named_parameters():
        g = (p.main_grad if getattr(p, "main_grad", None) is not None else p.grad).float()
        rel, cos = _stats(g, g32[n])
        rel_a, cos_a = _stats(gbf[n], g32[n])
        rows.append((n, rel, cos, rel_a, cos_a, g32[n].norm().item(), g.norm().item(), gbf[n].norm().item()))
    return {"loss": (loss.item(), lbf, l32), "rows": rows, "dims": {n: p.dim() for n, p in model.named_parameters()},
            "agg": (_stats(torch.cat([(p.main_grad if getattr(p, "main_grad", None) is not None else p.grad).float()
                                      .flatten() for _, p in model.named_parameters()]),
                           torch.cat([g32[n].flatten() for n, _ in model.named_parameters()])),
                    _stats(torch.cat([gbf[n].flatten() for n, _ in model.named_parameters()]),
                           torch.cat([g32[n].flatten() for n, _ in model.named_parameters()])))}


def summarize(res):
    rows = [r for r in res["rows"] if r[3] < 10]      # structurally-zero gradients (a bias under a BN) aside
    med = lambda v: sorted(v)[len(v) // 2]             # noqa: E731
    return {"loss_dph_aten_bf16_fp32": [round(v, 5) for v in res["loss"]],
            "agg_rel_dph": round(res["agg"][0][0], 4), "agg_rel_aten_bf16": round(res["agg"][1][0], 4),
            "median_rel_dph": round(med([r[1] for r in rows]), 4),
            "median_rel_aten_bf16": round(med([r[3] for r in rows]), 4),
            "max_rel_dph": round(max(r[1] for r in rows), 4), "max_rel_aten_bf16": round(max(r[3] for r in rows), 4),
            "min_cos_dph": round(min(r[2] for r in rows), 5), "min_cos_aten_bf16": round(min(r[4] for r in rows), 5),
            "n_params": len(res["rows"]), "n_zero_grad": len(res["rows"]) - len(rows),
            "worst": sorted(((r[0], round(r[1], 4), round(r[3], 4)) for r in rows), key=lambda t: -t[1])[:6]}


def _bf16_round_(model):
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return model


def _bn_shift_(model, beta):
    """Every BatchNorm's shift set to ``beta`` (None: keep 0): with beta = 3 the following ReLU clips ~0.1 % of the
    normalised activations instead of half, and the network stops amplifying rounding block over block."""
    from distributed_pytorch_hpc_amd.ops.batchnorm import BatchNormAct2d

    if beta is not None:
        with torch.no_grad():
            for mod in model.modules():
                if isinstance(mod, (BatchNormAct2d, torch.nn.BatchNorm2d)):
                    mod.bias.fill_(beta)
    return model


def resnet_rows(gamma=0.25, batch=32, res=112, beta=None):
    from distributed_pytorch_hpc_amd.models.resnet import Bottleneck, resnet50
    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ModuleWrapPolicy

    torch.manual_seed(0)
    m = resnet50(num_classes=1000).to(DEV).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, Bottleneck):
                mod.bn3.weight.fill_(gamma)
    _bf16_round_(_bn_shift_(m, beta))
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand(batch, 3, res, res, device=DEV, generator=g).to(torch.bfloat16).float()
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=DEV, generator=g)

    def wrap(model, mp):
        return FSDP(model, mixed_precision=mp, auto_wrap_policy=ModuleWrapPolicy({Bottleneck}))

    return _rows(m, x, lambda out: F.cross_entropy(out.float(), y), wrap)


def unet_rows(batch=2, h=96, w=184, beta=None):
    from distributed_pytorch_hpc_amd.models.unet import SimpleUNet, to_channels_last
    from distributed_pytorch_hpc_amd.ops.loss import latitude_weighted_mse
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP

    torch.manual_seed(0)
    m = _bf16_round_(_bn_shift_(to_channels_last(SimpleUNet(65, 65, 64).to(DEV)), beta))
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.randn(batch, 65, h, w, device=DEV, generator=g).to(torch.bfloat16).float()
    x = x.contiguous(memory_format=torch.channels_last)
    y = (x + 0.1 * torch.randn(x.shape, device=DEV, generator=g)).contiguous(memory_format=torch.channels_last)

    def wrap(model, mp):
        return DDP(model, mixed_precision=mp)

    return _rows(m, x, lambda out: latitude_weighted_mse(out.float(), y), wrap)


def _assert_close(res, absolute: bool, cos_floor: dict):
    """``absolute``: every parameter within rel 5e-2 / cosine 0.995 of fp32.  Always: each parameter's error within
    noise of stock bf16's, every conv / linear weight at cosine > 0.995 (``cos_floor`` overrides per name)."""
    s = summarize(res)
    print(s)
    ld, lb, l32 = res["loss"]
    gmax = max(r[5] for r in res["rows"])
    bad = []
    for n, rel, cos, rel_a, cos_a, n32, nd, na in res["rows"]:
        if rel_a >= 10:   # true gradient ~0 (bias under a BatchNorm): both bf16 paths return rounding noise
            ok = nd <= 3 * na + 1e-6 * gmax
        else:
            ok = rel <= (1.25 * rel_a + 2e-2 if rel_a < 0.1 else 1.5 * rel_a + 5e-2)
            if absolute:
                ok = ok and rel < 5e-2 and cos > 0.995
            if n.endswith("weight") and res["dims"][n] >= 2:
                ok = ok and cos > cos_floor.get(n, 0.995)
        if not ok:
            bad.append((n, rel, cos, rel_a, cos_a))
    assert abs(ld - l32) < 2e-3 * abs(l32), s
    assert not bad, "\n".join(f"{n}: rel {r:.3e} cos {c:.5f} (aten bf16: rel {ra:.3e} cos {ca:.5f})"
                               for n, r, c, ra, ca in bad[:20])
    assert s["agg_rel_dph"] < 1e-2 and s["agg_rel_dph"] <= 1.25 * s["agg_rel_aten_bf16"] + 1e-3, s


def test_resnet50_bf16_fsdp_gradients_match_fp32(dph_native):
    # per-parameter errors track stock bf16 MIOpen's (conv weights 0.04-0.08 rel, cosine >= 0.9968 for both, the
    # stem aside: its 3x3 max-pool routes gradients by bf16 ties, cosine 0.990 for both; profiles/r5/wholenet/)
    _assert_close(resnet_rows(gamma=1.0, beta=3.0), absolute=False, cos_floor={"conv1.weight": 0.985})


def test_simple_unet_bf16_ddp_gradients_match_fp32(dph_native):
    _assert_close(unet_rows(beta=3.0), absolute=True, cos_floor={})
