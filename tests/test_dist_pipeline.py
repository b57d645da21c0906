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


# ---------------------------------------------------------------------------------------------- schedule plans
def _exchanges(P, v, M):
    from distributed_pytorch_hpc_amd.parallel.pipeline import schedule_plan

    plans = [schedule_plan(P, v, M, r) for r in range(P)]
    ex = []
    for r in range(P):
        lst = []
        for op in plans[r]:
            if op[0] != "X":
                continue
            _, sf, sb, rp, rn = op
            s = []
            if sf:
                s.append(("send", (r + 1) % P, "act"))
            if sb:
                s.append(("send", (r - 1) % P, "grad"))
            if rp is not None:
                s.append(("recv", (r - 1) % P, "act"))
            if rn is not None:
                s.append(("recv", (r + 1) % P, "grad"))
            lst.append(s)
        ex.append(lst)
    return plans, ex


def _deadlock_free(P, v, M):
    """Each rank posts one grouped exchange at a time and moves on only when every op of it has met its peer's
    matching op (the i-th send on a directed channel <-> the i-th receive): the plan must always make progress."""
    _, ex = _exchanges(P, v, M)
    pos, cnt, cur = [0] * P, {}, [None] * P

    def post(r):
        if pos[r] >= len(ex[r]):
            cur[r] = None
            return
        ops = []
        for kind, peer, what in ex[r][pos[r]]:
            key = (r, peer, what) if kind == "send" else (peer, r, what)
            side = 0 if kind == "send" else 1
            c = cnt.setdefault(key, [0, 0])
            ops.append((key, side, c[side]))
            c[side] += 1
        cur[r] = ops

    for r in range(P):
        post(r)
    while any(c is not None for c in cur):
        moved = False
        for r in range(P):
            if cur[r] is not None and all(cnt[k][1 - s] > i for k, s, i in cur[r]):
                pos[r] += 1
                post(r)
                moved = True
        if not moved:
            return False
    return all(a == b for a, b in cnt.values())


def _dataflow_ok(P, v, M):
    """Every forward consumes exactly the previous virtual stage's activation of ITS micro-batch (every backward the
    next stage's gradient), in FIFO order per chunk, and nothing is left over."""
    from distributed_pytorch_hpc_amd.parallel.pipeline import chunk_of, microbatch_of

    plans, _ = _exchanges(P, v, M)
    sent = {}
    for r in range(P):
        out = dx = None
        for op in plans[r]:
            if op[0] == "F":
                out = (chunk_of(op[1], True, P, v) * P + r, microbatch_of(op[1], P, v))
            elif op[0] == "B":
                dx = (chunk_of(op[1], False, P, v) * P + r, microbatch_of(op[1], P, v))
            else:
                if op[1]:
                    sent.setdefault((r, (r + 1) % P, "act"), []).append(out)
                if op[2]:
                    sent.setdefault((r, (r - 1) % P, "grad"), []).append(dx)
    for r in range(P):
        fin, gin, cnt = [[] for _ in range(v)], [[] for _ in range(v)], {}
        for op in plans[r]:
            if op[0] in ("F", "B"):
                fwd = op[0] == "F"
                c, m = chunk_of(op[1], fwd, P, v), microbatch_of(op[1], P, v)
                if fwd and not (r == 0 and c == 0):
                    if not fin[c] or fin[c].pop(0) != (c * P + r - 1, m):
                        return False
                if not fwd and not (r == P - 1 and c == v - 1):
                    if not gin[c] or gin[c].pop(0) != (c * P + r + 1, m):
                        return False
            else:
                for idx, q, key in ((3, fin, ((r - 1) % P, r, "act")), (4, gin, ((r + 1) % P, r, "grad"))):
                    if op[idx] is not None:
                        i = cnt.get(key, 0)
                        cnt[key] = i + 1
                        q[op[idx]].append(sent[key][i])
        if any(fin) or any(gin):
            return False
    return True


def _channel_kinds_match(P, v, M):
    """RCCL / gloo match point-to-point messages per (src, dst) pair in issue order, whatever they carry: the i-th
    message rank a sends to rank b must be the i-th one b receives from a, of the same kind (activation / gradient)."""
    _, ex = _exchanges(P, v, M)
    sends, recvs = {}, {}
    for r in range(P):
        for grp in ex[r]:
            for kind, peer, what in grp:
                if kind == "send":
                    sends.setdefault((r, peer), []).append(what)
                else:
                    recvs.setdefault((peer, r), []).append(what)
    return sends == recvs


def test_schedule_plans_deadlock_free_and_consistent():
    for P in (2, 3, 4, 8):
        for v in (1, 2, 3, 4):
            if v > 1 and P < 3:
                continue
            for M in ([1, 2, 3, 5, 8, 16] if v == 1 else [P, 2 * P, 3 * P, 4 * P]):
                assert _channel_kinds_match(P, v, M), (P, v, M)
                assert _deadlock_free(P, v, M), (P, v, M)
                assert _dataflow_ok(P, v, M), (P, v, M)


def test_plan_counts():
    from distributed_pytorch_hpc_amd.parallel.pipeline import schedule_plan

    for P, v, M in ((4, 1, 8), (4, 2, 16), (3, 3, 6)):
        for r in range(P):
            ops = schedule_plan(P, v, M, r)
            assert sum(op[0] == "F" for op in ops) == M * v and sum(op[0] == "B" for op in ops) == M * v
    with pytest.raises(ValueError, match="divisible"):
        schedule_plan(4, 2, 6, 0)
    with pytest.raises(ValueError, match="at least 3"):
        schedule_plan(2, 2, 4, 0)


def test_partition_by_cost():
    from distributed_pytorch_hpc_amd.models.llama2 import get_preset
    from distributed_pytorch_hpc_amd.parallel.pipeline import llama_costs, partition_by_cost

    # a heavy head pulls layers off the last stage
    assert partition_by_cost([1.0] * 10, 3, 0.0, 2.5) == [(0, 4), (4, 8), (8, 10)]
    assert partition_by_cost([1.0] * 8, 4) == [(0, 2), (2, 4), (4, 6), (6, 8)]
    # Llama-2-7B: the head is ~0.6 of a block, so 8/8/8/8 stays optimal at whole-layer granularity
    blocks, emb, head = llama_costs(get_preset("llama2-7b"), 4096)
    assert 0.5 < head / blocks[0] < 0.8
    assert partition_by_cost(blocks, 4, emb, head) == [(0, 8), (8, 16), (16, 24), (24, 32)]
    # 26 layers / 4 stages: the last stage takes the short slice
    b = partition_by_cost(blocks[:26], 4, emb, head)
    assert [hi - lo for lo, hi in b][-1] == 6
    with pytest.raises(ValueError):
        partition_by_cost([1.0] * 3, 4)


PRESET8 = dict(PRESET, n_layers=8)


def _model8():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**PRESET8), device="cpu", dtype=torch.float32, seed=11)


def _reference8(m_micro):
    from distributed_pytorch_hpc_amd.parallel.pipeline import lm_loss

    m = _model8()
    x, y = _data(b=24)
    total = 0.0
    for xm, ym in zip(x.chunk(m_micro), y.chunk(m_micro)):
        loss = lm_loss(m(xm), ym) / m_micro
        loss.backward()
        total += loss.item()
    return total, {n: p.grad.clone() for n, p in m.named_parameters()}


def _interleaved_worker(rank, world, pp, v, m_micro, costs):
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, lm_loss, split_llama_virtual

    model = _model8()
    names = {id(p): n for n, p in model.named_parameters()}
    chunks = split_llama_virtual(model, pp, v, rank, costs=costs)
    sched = PipelineSchedule(chunks, rank, pp, m_micro, loss_fn=lm_loss, schedule="interleaved")
    x, y = _data(b=24)
    out = []
    for _ in range(2):   # second step: cached boundary shape, no header
        for p in chunks.parameters():
            p.grad = None
        losses = sched.step(inputs=x if rank == 0 else None, target=y if rank == pp - 1 else None)
        out.append([float(l) for l in losses])
    grads = {names[id(p)]: p.grad.clone() for p in chunks.parameters()}
    # forward-only pass through the same chunks
    logits = sched.forward(x if rank == 0 else None)
    return out, grads, (logits is not None), sched.bubble


@pytest.mark.parametrize("pp,v,m_micro", [(3, 2, 3), (3, 2, 6), (4, 2, 4), (4, 2, 8)])
def test_interleaved_matches_single_process(pp, v, m_micro):
    ref_loss, ref_g = _reference8(m_micro)
    costs = None
    if pp * v == 8:
        costs = ([1.0] * 8, 0.0, 0.0)   # one layer per virtual stage
    outs = run_distributed(_interleaved_worker, pp, pp, v, m_micro, costs)
    seen = set()
    for r, (steps, grads, has_logits, bub) in enumerate(outs):
        assert has_logits == (r == pp - 1)
        assert abs(bub - (pp - 1) / (v * m_micro + pp - 1)) < 1e-12
        for n, g in grads.items():
            assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), (r, n)
            seen.add(n)
    assert seen == set(ref_g)
    for step_losses in outs[pp - 1][0]:
        assert len(step_losses) == m_micro and abs(sum(step_losses) / m_micro - ref_loss) < 1e-5


def _varying_shape_worker(rank, world, pp, v, schedule, m_micro):
    from distributed_pytorch_hpc_amd.parallel.pipeline import (PipelineSchedule, lm_loss, split_llama,
                                                                split_llama_virtual)

    model = _model8()
    names = {id(p): n for n, p in model.named_parameters()}
    chunks = split_llama_virtual(model, pp, v, rank) if v > 1 else split_llama(model, pp, rank)
    sched = PipelineSchedule(chunks, rank, pp, m_micro, loss_fn=lm_loss, schedule=schedule)
    out = []
    for s in (16, 8, 24):   # sequence length changes every step: each call must re-announce the boundary shape
        x, y = _data(b=12, s=s)
        for p in chunks.parameters():
            p.grad = None
        losses = sched.step(inputs=x if rank == 0 else None, target=y if rank == pp - 1 else None)
        out.append(([float(l) for l in losses], {names[id(p)]: p.grad.clone() for p in chunks.parameters()}))
    # forward-only pass at yet another length
    x, _ = _data(b=12, s=12)
    logits = sched.forward(x if rank == 0 else None)
    return out, None if logits is None else tuple(logits.shape)


@pytest.mark.parametrize("pp,v,schedule", [(2, 1, "1f1b"), (3, 2, "interleaved")])
def test_pipeline_shape_changes_between_steps(pp, v, schedule):
    """Advisor r4: the boundary shape header was sent once per schedule object, so a later step with another
    sequence length posted receive buffers of the old shape.  Every step must match its own single-process run."""
    from distributed_pytorch_hpc_amd.parallel.pipeline import lm_loss

    m_micro = 3
    outs = run_distributed(_varying_shape_worker, pp, pp, v, schedule, m_micro)
    for step, s in enumerate((16, 8, 24)):
        m = _model8()
        x, y = _data(b=12, s=s)
        total = 0.0
        for xm, ym in zip(x.chunk(m_micro), y.chunk(m_micro)):
            loss = lm_loss(m(xm), ym) / m_micro
            loss.backward()
            total += loss.item()
        ref_g = {n: p.grad for n, p in m.named_parameters()}
        last_losses = outs[pp - 1][0][step][0]
        assert abs(sum(last_losses) / m_micro - total) < 1e-5, (step, s)
        for r in range(pp):
            for n, g in outs[r][0][step][1].items():
                assert torch.allclose(g, ref_g[n], atol=1e-5, rtol=1e-4), (step, r, n)
    assert outs[pp - 1][1] is not None and outs[pp - 1][1][1] == 12
