"""gloo parity of pipeline parallelism (GPipe / 1F1B, PP x DP) against a single-process step."""
import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed

PRESET = dict(dim=64, n_layers=4, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)


def _model():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=11)


def _data(b=8, s=16):
    g = torch.Generator().manual_seed(5)
    t = torch.randint(0, PRESET["vocab_size"], (b, s + 1), generator=g)
    return t[:, :-1], t[:, 1:]


def _reference(m_micro=4):
    from distributed_pytorch_hpc_amd.parallel.pipeline import lm_loss

    m = _model()
    x, y = _data()
    total = 0.0
    for xm, ym in zip(x.chunk(m_micro), y.chunk(m_micro)):
        loss = lm_loss(m(xm), ym) / m_micro
        loss.backward()
        total += loss.item()
    return total, {n: p.grad.clone() for n, p in m.named_parameters()}


def _pp_worker(rank, world, pp, schedule, m_micro):
    from distributed_pytorch_hpc_amd.comm.mesh import Mesh
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, lm_loss, split_llama

    dp = world // pp
    mesh = Mesh((dp, pp), ("dp", "pp"))
    stage = mesh.local_rank("pp")
    model = _model()
    names = {id(p): n for n, p in model.named_parameters()}
    sm = split_llama(model, pp, stage)
    sched = PipelineSchedule(sm, stage, pp, m_micro, loss_fn=lm_loss, group=mesh.group("pp"), schedule=schedule)
    x, y = _data()
    xl, yl = x.chunk(dp)[mesh.local_rank("dp")], y.chunk(dp)[mesh.local_rank("dp")]
    losses = sched.step(inputs=xl if stage == 0 else None, target=yl if stage == pp - 1 else None)
    grads = {}
    for p in sm.parameters():
        g = p.grad.clone()
        if dp > 1:
            dist.all_reduce(g, group=mesh.group("dp"))
            g /= dp
        grads[names[id(p)]] = g
    return [float(l) for l in losses], grads


@pytest.mark.parametrize("schedule", ["gpipe", "1f1b"])
def test_pipeline_2stage_matches_single_process(schedule):
    ref_loss, ref_g = _reference()
    outs = run_distributed(_pp_worker, 2, 2, schedule, 4)
    last_losses = outs[1][0]
    assert abs(sum(last_losses) / 4 - ref_loss) < 1e-5
    for _, grads in outs:
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), n


def test_pipeline_4stage_1f1b():
    ref_loss, ref_g = _reference()
    outs = run_distributed(_pp_worker, 4, 4, "1f1b", 4)
    assert abs(sum(outs[3][0]) / 4 - ref_loss) < 1e-5
    for _, grads in outs:
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), n


def test_pp2_x_dp2():
    # each dp replica pipelines half the batch in 2 micro-batches: same micro-batch partition as 4 overall
    ref_loss, ref_g = _reference()
    outs = run_distributed(_pp_worker, 4, 2, "1f1b", 2)
    for _, grads in outs:
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), n


def test_bubble_math():
    from distributed_pytorch_hpc_amd.parallel.pipeline import bubble_fraction

    assert abs(bubble_fraction(4, 4) - 3 / 7) < 1e-12
    assert bubble_fraction(1, 8) == 0.0


def test_uneven_microbatches_rejected_before_any_transfer():
    """Only micro-batch 0 carries a shape header: a batch not divisible by n_microbatches must fail on the
    stage that holds it, before any send (single stage, no process group)."""
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule

    sched = PipelineSchedule(torch.nn.Linear(4, 4), 0, 1, 4, loss_fn=lambda y, t: (y - t).pow(2).mean(),
                             device=torch.device("cpu"))
    with pytest.raises(ValueError, match="not divisible"):
        sched.step(inputs=torch.randn(6, 4), target=torch.randn(6, 4))
    with pytest.raises(ValueError, match="not divisible"):
        sched.forward(torch.randn(2, 4))
    assert len(sched.step(inputs=torch.randn(8, 4), target=torch.randn(8, 4))) == 4
