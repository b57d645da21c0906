"""World-8 gloo parity of the exact BASELINE.json meshes against one process with the same global batch:
TP=8 (+SP, loss-parallel), FSDP(2) x TP(4), PP4 x DDP2 (1F1B), CP=8 ring (zig-zag) and Ulysses, ResNet FSDP over 8
ranks, plus every configs/llama2_7b_*.yaml launched through scripts/run_config.py at world 8 with a tiny model.

The 8-GPU node only exists at the round-end driver run; these tests rehearse its rank layouts on CPU so a mesh
bug (wrong group, wrong shard, wrong schedule) fails here first.  Reference: fsdp_tp/fsdp_tp_example.py:103-187,
scripts/06_hybrid_parallelism/01_fsdp_tp_hybrid.py:73-155, scripts/04_pipeline_parallel_pp/03_pipeline_training.py.
"""
import math
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 2
# heads, FFN (352), vocab and sequence divisible by 8: every BASELINE mesh shards it evenly
PRESET8 = dict(dim=128, n_layers=4, n_heads=8, vocab_size=128, max_seq_len=64, multiple_of=32)


def _model():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**PRESET8), device="cpu", dtype=torch.float32, seed=7)


def _batches(global_b=8, s=16):
    g = torch.Generator().manual_seed(3)
    return [torch.randint(0, PRESET8["vocab_size"], (global_b, s + 1), generator=g) for _ in range(STEPS)]


def _reference():
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    m = _model()
    eng = DataParallelEngine(m, shard=False)
    eng.configure_optimizer(OptimConfig(lr=1e-2, weight_decay=0.1))
    losses = []
    for t in _batches():
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        eng.step()
        eng.zero_grad()
        losses.append(loss.item())
    return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}


# ---------------------------------------------------------------------------------------------- TP / hybrid
def _tp_worker(rank, world, dp):
    from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama

    mesh = DeviceMesh2D(dp, world // dp)
    m = _model()
    parallelize_llama(m, mesh.tp_group, sequence_parallel=True, loss_parallel=True)
    eng = DataParallelEngine(m, process_group=mesh.dp_group, shard=dp > 1, bucket_cap_mb=0.05)
    eng.configure_optimizer(OptimConfig(lr=1e-2, weight_decay=0.1))
    losses = []
    for t in _batches():
        local = t.chunk(dp, 0)[mesh.dp_rank]
        loss = m(local[:, :-1], local[:, 1:])
        loss.backward()
        eng.step()
        eng.zero_grad()
        lt = loss.detach().clone()
        dist.all_reduce(lt, group=mesh.dp_group)
        losses.append(lt.item() / dp)
    eng.synchronize()
    return losses, mesh.tp_rank, {k: v.detach().clone() for k, v in m.state_dict().items()}


def _check_tp(ref, outs, tp, tol=5e-5):
    ref_losses, ref_sd = ref
    for losses, _, _ in outs:
        for a, b in zip(ref_losses, losses):
            assert abs(a - b) < tol * max(1.0, abs(a)), (ref_losses, losses)
    by_tp = {r: sd for _, r, sd in outs}
    for layer in range(PRESET8["n_layers"]):
        w2 = torch.cat([by_tp[r][f"layers.{layer}.feed_forward.w2.weight"] for r in range(tp)], 1)
        assert torch.allclose(w2, ref_sd[f"layers.{layer}.feed_forward.w2.weight"], atol=tol), layer
        wo = torch.cat([by_tp[r][f"layers.{layer}.attention.wo.weight"] for r in range(tp)], 1)
        assert torch.allclose(wo, ref_sd[f"layers.{layer}.attention.wo.weight"], atol=tol), layer
    emb = torch.cat([by_tp[r]["tok_embeddings.weight"] for r in range(tp)], 0)
    assert torch.allclose(emb, ref_sd["tok_embeddings.weight"], atol=tol)
    out = torch.cat([by_tp[r]["output.weight"] for r in range(tp)], 0)
    assert torch.allclose(out, ref_sd["output.weight"], atol=tol)
    assert torch.allclose(by_tp[0]["norm.weight"], ref_sd["norm.weight"], atol=tol)


def test_tp8_sp_loss_parallel_matches_single_process():
    """BASELINE config 3: TP = 8 (column / row shards, sequence-parallel norms, vocab-parallel loss)."""
    _check_tp(_reference(), run_distributed(_tp_worker, 8, 1, timeout=400), 8)


def test_fsdp2_x_tp4_matches_single_process():
    """BASELINE config 4: the (dp=2, tp=4) mesh, sharded optimizer over dp."""
    _check_tp(_reference(), run_distributed(_tp_worker, 8, 2, timeout=400), 4)


# ---------------------------------------------------------------------------------------------- PP x DP
def _lm_ref_grads(m_micro):
    from distributed_pytorch_hpc_amd.parallel.pipeline import lm_loss

    m = _model()
    t = _batches()[0]
    x, y = t[:, :-1], t[:, 1:]
    total = 0.0
    for xm, ym in zip(x.chunk(m_micro), y.chunk(m_micro)):
        loss = lm_loss(m(xm), ym) / m_micro
        loss.backward()
        total += loss.item()
    return total, {n: p.grad.clone() for n, p in m.named_parameters()}


def _pp_worker(rank, world, pp, m_micro):
    from distributed_pytorch_hpc_amd.comm.mesh import Mesh
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, lm_loss, split_llama

    dp = world // pp
    mesh = Mesh((pp, dp), ("pp", "dp"))     # the layout of bench.py --layout pp / three_d_parallel.py
    stage, dpr = mesh.local_rank("pp"), mesh.local_rank("dp")
    model = _model()
    names = {id(p): n for n, p in model.named_parameters()}
    sm = split_llama(model, pp, stage)
    eng = DataParallelEngine(sm, mesh.group("dp"), shard=False, bucket_cap_mb=0.05)
    sched = PipelineSchedule(sm, stage, pp, m_micro, loss_fn=lm_loss, group=mesh.group("pp"), schedule="1f1b",
                             dp_engine=eng)
    t = _batches()[0]
    x, y = t[:, :-1].chunk(dp)[dpr], t[:, 1:].chunk(dp)[dpr]
    losses = sched.step(inputs=x if stage == 0 else None, target=y if stage == pp - 1 else None)
    eng.synchronize()
    # the engine reduced SUMs over dp into main_grad; the mean is what the reference holds
    grads = {names[id(p)]: p.main_grad.detach().clone() / dp for p in sm.parameters()}
    return [float(v) for v in losses], stage, grads


def test_pp4_x_ddp2_1f1b_matches_single_process():
    """BASELINE config 5: 4 stages x DDP 2, 1F1B, gradients reduced over dp on the last micro-batch.  Each dp
    replica pipelines half the batch in 2 micro-batches: the same 4-way micro-batch partition as the reference."""
    ref_loss, ref_g = _lm_ref_grads(4)
    outs = run_distributed(_pp_worker, 8, 4, 2, timeout=400)
    seen = set()
    for losses, stage, grads in outs:
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), (stage, n)
            seen.add(n)
    assert seen == set(ref_g)                    # every parameter lives on some stage
    last = [v for lo, st, _ in outs if st == 3 for v in lo]   # 2 replicas x 2 micro-batch losses
    assert len(last) == 4 and abs(sum(last) / 4 - ref_loss) < 1e-5


def _model_l8():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**dict(PRESET8, n_layers=8)), device="cpu", dtype=torch.float32, seed=7)


def _ipp_worker(rank, world, pp, v, m_micro):
    from distributed_pytorch_hpc_amd.comm.mesh import Mesh
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, lm_loss, split_llama_virtual

    dp = world // pp
    mesh = Mesh((pp, dp), ("pp", "dp"))
    stage, dpr = mesh.local_rank("pp"), mesh.local_rank("dp")
    model = _model_l8()
    names = {id(p): n for n, p in model.named_parameters()}
    chunks = split_llama_virtual(model, pp, v, stage)
    engines = [DataParallelEngine(c, mesh.group("dp"), shard=False, bucket_cap_mb=0.05) for c in chunks]
    sched = PipelineSchedule(chunks, stage, pp, m_micro, loss_fn=lm_loss, group=mesh.group("pp"),
                             schedule="interleaved", dp_engine=engines)
    t = _batches(global_b=16)[0]
    x, y = t[:, :-1].chunk(dp)[dpr], t[:, 1:].chunk(dp)[dpr]
    losses = sched.step(inputs=x if stage == 0 else None, target=y if stage == pp - 1 else None)
    grads = {}
    for e, c in zip(engines, chunks):
        e.synchronize()
        grads.update({names[id(p)]: p.main_grad.detach().clone() / dp for p in c.parameters()})
    return [float(l) for l in losses], stage, grads, sched.bubble


def test_pp4_x_ddp2_interleaved_matches_single_process():
    """BASELINE config 5 with the interleaved schedule: 4 ranks x 2 model chunks of one layer each, one
    data-parallel engine per chunk (each chunk's gradients reduce at its own last backward), 8 micro-batches per dp
    replica -- the same micro-batch partition (16 of 1 sequence) as the single-process reference."""
    from distributed_pytorch_hpc_amd.parallel.pipeline import lm_loss

    m = _model_l8()
    t = _batches(global_b=16)[0]
    x, y = t[:, :-1], t[:, 1:]
    ref_loss = 0.0
    for xm, ym in zip(x.chunk(16), y.chunk(16)):
        loss = lm_loss(m(xm), ym) / 16
        loss.backward()
        ref_loss += loss.item()
    ref_g = {n: p.grad.clone() for n, p in m.named_parameters()}
    outs = run_distributed(_ipp_worker, 8, 4, 2, 8, timeout=400)
    seen = set()
    for losses, stage, grads, bub in outs:
        assert abs(bub - 3 / (2 * 8 + 3)) < 1e-12
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), (stage, n)
            seen.add(n)
    assert seen == set(ref_g)
    last = [v for lo, st, _, _ in outs if st == 3 for v in lo]
    assert len(last) == 16 and abs(sum(last) / 16 - ref_loss) < 1e-5


# ---------------------------------------------------------------------------------------------- CP = 8
def _qkv(b=1, s=64, h=8, d=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(b, s, h, d, generator=g) for _ in range(3)]


def _ring_worker(rank, world):
    from distributed_pytorch_hpc_amd.parallel.context_parallel import ring_attention, shard_sequence

    q, k, v = _qkv()
    g = torch.Generator().manual_seed(9)
    do = torch.randn(q.shape, generator=g)
    grp = dist.group.WORLD
    ql, kl, vl = (shard_sequence(t, grp, "zigzag").requires_grad_() for t in (q, k, v))
    o = ring_attention(ql, kl, vl, grp, causal=True, layout="zigzag")
    o.backward(shard_sequence(do, grp, "zigzag"))
    return o.detach(), ql.grad, kl.grad, vl.grad


def test_cp8_zigzag_ring_matches_full_attention():
    from distributed_pytorch_hpc_amd.ops.attention import attention_reference
    from distributed_pytorch_hpc_amd.parallel.context_parallel import unshard_sequence

    q, k, v = (t.clone().requires_grad_() for t in _qkv())
    o = attention_reference(q, k, v, True, 1 / math.sqrt(q.shape[-1]))
    g = torch.Generator().manual_seed(9)
    o.backward(torch.randn(o.shape, generator=g))
    outs = run_distributed(_ring_worker, 8, timeout=400)
    for i, ref in enumerate((o.detach(), q.grad, k.grad, v.grad)):
        got = unshard_sequence([out[i] for out in outs], "zigzag")
        assert torch.allclose(got, ref, atol=2e-5), (i, (got - ref).abs().max())


def _llama_cp_worker(rank, world, mode, layout):
    from distributed_pytorch_hpc_amd.parallel.context_parallel import apply_context_parallel, shard_sequence

    m = _model()
    apply_context_parallel(m, dist.group.WORLD, mode, layout=layout)
    t = _batches(global_b=2, s=64)[0]
    x = shard_sequence(t[:, :-1], dist.group.WORLD, layout)
    y = shard_sequence(t[:, 1:], dist.group.WORLD, layout)
    loss = m(x, y)
    loss.backward()
    gw = m.layers[0].attention.wqkv.weight.grad.clone()
    dist.all_reduce(gw)
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    return lt.item() / world, gw / world


@pytest.mark.parametrize("mode,layout", [("ulysses", "contiguous"), ("ring", "zigzag")])
def test_llama_cp8_matches_single_process(mode, layout):
    """CP = 8 inside the Llama (Ulysses all-to-all over 8 heads; zig-zag ring): loss and wqkv gradient."""
    m = _model()
    t = _batches(global_b=2, s=64)[0]
    loss = m(t[:, :-1], t[:, 1:])
    loss.backward()
    ref_g = m.layers[0].attention.wqkv.weight.grad
    for lt, gw in run_distributed(_llama_cp_worker, 8, mode, layout, timeout=400):
        assert abs(lt - loss.item()) < 1e-5
        assert torch.allclose(gw, ref_g, atol=1e-5, rtol=1e-4)


# ---------------------------------------------------------------------------------------------- ResNet FSDP W = 8
def _resnet_setup():
    from distributed_pytorch_hpc_amd.models import resnet
    from distributed_pytorch_hpc_amd.models.resnet import BasicBlock

    torch.manual_seed(4)
    m = resnet("resnet18", num_classes=10, cifar_stem=True)
    m.eval()   # BatchNorm on running statistics: the per-rank batch statistics would otherwise differ by design
    return m, BasicBlock


def _resnet_data():
    g = torch.Generator().manual_seed(12)
    return torch.randn(16, 3, 16, 16, generator=g), torch.randint(0, 10, (16,), generator=g)


def _resnet_fsdp_worker(rank, world):
    import torch.nn.functional as F

    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ModuleWrapPolicy

    m, block = _resnet_setup()
    f = FSDP(m, auto_wrap_policy=ModuleWrapPolicy({block}))
    opt = f.make_optimizer("sgd", lr=0.1, momentum=0.9, weight_decay=1e-4)
    x, y = _resnet_data()
    for _ in range(STEPS):
        opt.zero_grad()
        F.cross_entropy(f(x.chunk(world)[rank]), y.chunk(world)[rank]).backward()
        opt.step()
    f.engine.synchronize()
    return f.full_state_dict(rank0_only=False)


def test_resnet_fsdp_world8_matches_single_process():
    """BASELINE config 2's strategy (FULL_SHARD per residual block) over 8 ranks."""
    import torch.nn.functional as F

    from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP

    m, _ = _resnet_setup()
    d = DDP(m)
    opt = d.make_optimizer("sgd", lr=0.1, momentum=0.9, weight_decay=1e-4)
    x, y = _resnet_data()
    for _ in range(STEPS):
        opt.zero_grad()
        F.cross_entropy(d(x), y).backward()
        opt.step()
    ref = {k: v.detach().clone() for k, v in m.state_dict().items()}
    outs = run_distributed(_resnet_fsdp_worker, 8, timeout=400)
    for sd in outs:
        for k, v in ref.items():
            if k in sd and v.is_floating_point():
                assert torch.allclose(sd[k], v, atol=1e-5, rtol=1e-4), k


# ---------------------------------------------------------------------------------------------- the 7B configs
def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("cfg,extra", [
    ("llama2_7b_tp8.yaml", ["--device", "cpu", "--model", "tiny8", "--seq-len", "64", "--batch", "4", "--iters", "2"]),
    ("llama2_7b_fsdp2_tp4.yaml", ["--device", "cpu", "--model", "tiny8", "--seq-len", "64", "--batch", "4",
                                  "--iters", "2"]),
    ("llama2_7b_pp4_ddp2.yaml", ["--device", "cpu", "--model", "tiny8", "--seq-len", "64", "--batch", "8",
                                 "--microbatches", "4", "--iters", "2"]),
    ("llama2_7b_fsdp_bench.yaml", ["--device", "cpu", "--model", "tiny8", "--seq-len", "64", "--micro-batch", "2",
                                   "--steps", "1", "--warmup", "1"]),
])
def test_run_config_llama2_7b_world8(cfg, extra, tmp_path):
    """Every Llama-2-7B BASELINE config file runs end to end at world 8 (gloo) with the 7B model swapped for a tiny
    one -- the same launcher, driver, flags and mesh the 8-GPU node gets."""
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "run_config.py"), os.path.join(ROOT, "configs", cfg),
           "--nproc", "8", "--"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert any(ln.startswith("{") for ln in p.stdout.splitlines()), p.stdout[-2000:]


def _sp_count_worker(rank, world):
    from distributed_pytorch_hpc_amd.comm import functional as cf
    from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama

    mesh = DeviceMesh2D(1, world)
    m = _model()
    parallelize_llama(m, mesh.tp_group, sequence_parallel=True, loss_parallel=True)
    eng = DataParallelEngine(m, process_group=mesh.dp_group, shard=False, bucket_cap_mb=0.05)
    eng.configure_optimizer(OptimConfig(lr=1e-2))
    calls = {"hook": 0, "batched": 0}
    real_ar, real_batched = cf.all_reduce_, eng._reduce_tp_partial

    def counting_hook_ar(t, g, **kw):
        if t.shape == (PRESET8["dim"],) and not kw:   # a norm weight's gradient
            calls["hook"] += 1
        return real_ar(t, g, **kw)

    def counting_batched():
        calls["batched"] += 1
        return real_batched()

    cf.all_reduce_ = counting_hook_ar
    eng._reduce_tp_partial = counting_batched
    try:
        t = _batches()[0][:, :13]   # 8 x 12 tokens: divisible by tp, and 96 != dim
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        eng.step()
    finally:
        cf.all_reduce_ = real_ar
    assert len(eng._tp_partial) == 1
    n_sp = sum(1 for p in m.parameters() if getattr(p, "_dph_sequence_parallel", False))
    return calls, n_sp


def test_sp_norm_grads_one_batched_all_reduce():
    """With the data-parallel engine owning them, the sequence-parallel norm weights' TP-partial gradients cost ONE
    all-reduce per step (engine.step), not one per parameter from a backward hook."""
    outs = run_distributed(_sp_count_worker, 4)
    for calls, n_sp in outs:
        assert n_sp == 2 * PRESET8["n_layers"] + 1
        assert calls == {"hook": 0, "batched": 1}, calls
