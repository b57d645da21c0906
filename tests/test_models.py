"""Model zoo: parameter counts against the reference and CPU forward/backward shapes."""
import torch

from distributed_pytorch_hpc_amd import models


def n_params(m):
    return sum(p.numel() for p in m.parameters())


def test_llama_param_counts():
    assert models.get_preset("toy").num_params() == 18_089_216
    assert models.get_preset("llama2-7b").num_params() == 6_738_415_616
    m = models.build_llama("toy", device="cpu", dtype=torch.float32)
    assert n_params(m) == 18_089_216
    assert models.get_preset("llama2-7b").ffn_hidden == 11008


def test_unet_vit_pp_param_counts():
    assert n_params(models.SimpleUNet(65, 65)) == 7_742_849
    assert n_params(models.SimpleViT(65, 65, 8, 64, 128)) == 6_906_176
    assert n_params(models.PipelineTransformer()) == 11_700_736
    assert n_params(models.FourBlockMLP()) == 1_050_624


def test_resnet_param_counts():
    assert n_params(models.resnet50()) == 25_557_032
    assert n_params(models.resnet18()) == 11_689_512
    assert n_params(models.resnet18(num_classes=10, cifar_stem=True)) == 11_173_962


def test_forward_shapes_cpu():
    x = torch.randn(1, 65, 37, 72)
    assert models.SimpleUNet(65, 65, base_dim=8)(x).shape == x.shape   # odd latitude (reference X: 181)
    v = models.SimpleViT(65, 65, 8, 64, 128, embed_dim=64, depth=2, num_heads=4)
    assert v(torch.randn(2, 65, 64, 128)).shape == (2, 65, 64, 128)
    pp = models.PipelineTransformer(vocab_size=100, dim=32, n_heads=4, layers_per_stage=1)
    t = torch.randint(0, 100, (2, 16))
    assert pp(t).shape == (2, 16, 100)
    st = pp.stage_modules(2)
    assert st[1](st[0](t)).shape == (2, 16, 100)
    r = models.resnet18(num_classes=10, cifar_stem=True)
    out = r(torch.randn(2, 3, 32, 32))
    out.sum().backward()
    assert out.shape == (2, 10)


def test_llama_logits_and_loss_consistent():
    m = models.build_llama("tiny", device="cpu", dtype=torch.float32)
    t = torch.randint(0, 512, (2, 17))
    logits = m(t[:, :-1])
    loss = m(t[:, :-1], t[:, 1:])
    ref = torch.nn.functional.cross_entropy(logits.reshape(-1, 512), t[:, 1:].reshape(-1))
    assert torch.allclose(loss, ref, atol=1e-5)


def test_reference_state_dict_conversion():
    args = models.get_preset("tiny")
    m = models.build_llama(args, device="cpu", dtype=torch.float32)
    sd = m.state_dict()
    ref = {}
    hd = args.head_dim
    for k, v in sd.items():
        if "wqkv" in k:
            q, kk, vv = v.split([args.n_heads * hd, args.kv_heads * hd, args.kv_heads * hd])
            ref[k.replace("wqkv", "wq")], ref[k.replace("wqkv", "wk")], ref[k.replace("wqkv", "wv")] = q, kk, vv
        elif "w13" in k:
            a, b = v.chunk(2)
            ref[k.replace("w13", "w1")], ref[k.replace("w13", "w3")] = a, b
        else:
            ref[k] = v
    back = models.convert_reference_state_dict(ref, args)
    assert back.keys() == sd.keys()
    for k in sd:
        assert torch.equal(back[k], sd[k])


def test_bn_act_module_cpu_matches_batchnorm():
    """BatchNormAct2d on CPU == BatchNorm2d (+ residual) (+ ReLU), incl. running stats and eval."""
    from torch import nn
    from distributed_pytorch_hpc_amd.ops import BatchNormAct2d

    torch.manual_seed(0)
    for act in (True, False):
        fused, ref = BatchNormAct2d(16, act=act), nn.BatchNorm2d(16)
        with torch.no_grad():
            fused.weight.normal_(1, 0.3)
            fused.bias.normal_(0, 0.3)
        ref.load_state_dict(fused.state_dict())
        x, r = torch.randn(4, 16, 6, 6), torch.randn(4, 16, 6, 6)
        want = ref(x) + r
        want = torch.relu(want) if act else want
        torch.testing.assert_close(fused(x, r), want)
        torch.testing.assert_close(fused.running_mean, ref.running_mean)
        fused.eval(), ref.eval()
        want = torch.relu(ref(x)) if act else ref(x)
        torch.testing.assert_close(fused(x), want)


def test_resnet_state_dict_keys_torchvision_compatible():
    keys = set(models.resnet18().state_dict())
    assert "bn1.running_var" in keys and "layer2.0.downsample.1.weight" in keys
    assert not any("relu" in k for k in keys)
    assert len(keys) == 122


def test_vit_patch_embed_gemm_matches_conv():
    from distributed_pytorch_hpc_amd.models.vit import PatchEmbed

    torch.manual_seed(0)
    m = PatchEmbed(65, 64, 8)
    for shape in [(2, 65, 64, 128), (1, 65, 67, 130)]:
        x = torch.randn(shape)
        torch.testing.assert_close(m(x), m.proj(x).flatten(2).transpose(1, 2), rtol=1e-5, atol=1e-5)


def test_latitude_weighted_mse_cpu_reference():
    from distributed_pytorch_hpc_amd.ops.loss import latitude_weighted_mse, latitude_weights

    p, t = torch.randn(2, 3, 181, 36), torch.randn(2, 3, 181, 36)
    w = latitude_weights(181).view(1, 1, -1, 1)
    torch.testing.assert_close(latitude_weighted_mse(p, t), (w * (p - t) ** 2).mean())
    # equal latitude shards average to the global loss
    parts = [latitude_weighted_mse(p[:, :, i:i + 60], t[:, :, i:i + 60], 180, i) for i in (0, 60, 120)]
    pg, tg = p[:, :, :180], t[:, :, :180]
    wg = latitude_weights(180).view(1, 1, -1, 1)
    torch.testing.assert_close(sum(parts) / 3, (wg * (pg - tg) ** 2).mean())


def test_unet_block_output_slot_handoff_cpu(monkeypatch):
    """ConvBlock.out_slot: the second BatchNorm's slot goes to exactly one taker of exactly that output tensor, and
    DPH_UNET_OUT_FOLD=0 withholds it.  On the CPU SimpleUNet's gradients are identical with and without the skip
    slots (they arm only on the GPU kernel paths)."""
    from distributed_pytorch_hpc_amd.models.unet import SimpleUNet, conv_block
    from distributed_pytorch_hpc_amd.ops.conv import BnGradSlot

    torch.manual_seed(0)
    blk = conv_block(8, 16).train()
    x = torch.randn(2, 8, 6, 10)
    y = blk(x)
    other = y.clone()
    assert blk.out_slot(other) is None          # a different tensor: no slot (and the offer is withdrawn)
    y = blk(x)
    s = blk.out_slot(y)
    assert isinstance(s, BnGradSlot)
    assert blk.out_slot(y) is None              # taken once
    monkeypatch.setenv("DPH_UNET_OUT_FOLD", "0")
    y = blk(x)
    assert blk.out_slot(y) is None
    monkeypatch.delenv("DPH_UNET_OUT_FOLD")

    net = SimpleUNet(3, 3, 8).train()
    inp = torch.randn(2, 3, 12, 20)
    g = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("DPH_UNET_SKIP_FOLD", fold)
        net.zero_grad(set_to_none=True)
        net(inp).square().mean().backward()
        g[fold] = [p.grad.clone() for p in net.parameters()]
    for a, b in zip(g["1"], g["0"]):
        assert torch.equal(a, b)
