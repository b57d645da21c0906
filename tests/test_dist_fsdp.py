"""FSDP strategies (FULL_SHARD per-block / size policy, HYBRID, SHARD_GRAD_OP, NO_SHARD) vs one process (gloo)."""
import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed

PRESET = dict(dim=64, n_layers=3, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)
STEPS = 3


def _model():
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=21)


def _batches():
    g = torch.Generator().manual_seed(4)
    return [torch.randint(0, 128, (4, 17), generator=g) for _ in range(STEPS)]


def _reference():
    m = _model()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.1)
    losses = []
    for t in _batches():
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}


def _worker(rank, world, strategy, policy_kind):
    from distributed_pytorch_hpc_amd.models.llama2 import TransformerBlock
    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ModuleWrapPolicy, size_based_auto_wrap_policy

    m = _model()
    policy = {"block": ModuleWrapPolicy({TransformerBlock}), "size": size_based_auto_wrap_policy(5000),
              None: None}[policy_kind]
    kw = {}
    if strategy == "HYBRID_SHARD":
        g0 = dist.new_group([0, 1])
        g1 = dist.new_group([2, 3])
        r0 = dist.new_group([0, 2])
        r1 = dist.new_group([1, 3])
        kw = dict(process_group=g0 if rank < 2 else g1, replicate_group=r0 if rank % 2 == 0 else r1)
    f = FSDP(m, sharding_strategy=strategy, auto_wrap_policy=policy, bucket_cap_mb=0.02, **kw)
    opt = f.make_optimizer("adamw", lr=1e-2, weight_decay=0.1)
    losses = []
    for t in _batches():
        local = t.chunk(world, 0)[rank]
        loss = f(local[:, :-1], local[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        lt = loss.detach().clone()
        dist.all_reduce(lt)
        losses.append(lt.item() / world)
    sd = f.full_state_dict(rank0_only=False)
    return losses, sd


@pytest.mark.parametrize("strategy,policy", [("FULL_SHARD", "block"), ("FULL_SHARD", "size"),
                                             ("SHARD_GRAD_OP", None), ("NO_SHARD", None)])
def test_fsdp_strategies_match_single_process(strategy, policy):
    ref_losses, ref_sd = _reference()
    outs = run_distributed(_worker, 2, strategy, policy)
    for losses, sd in outs:
        for a, b in zip(ref_losses, losses):
            assert abs(a - b) < 3e-5 * max(1, abs(a)), (ref_losses, losses)
        for k, v in ref_sd.items():
            assert torch.allclose(v, sd[k], atol=3e-5), k


def test_hybrid_shard_4ranks():
    ref_losses, ref_sd = _reference()
    outs = run_distributed(_worker, 4, "HYBRID_SHARD", "block")
    for losses, sd in outs:
        for a, b in zip(ref_losses, losses):
            assert abs(a - b) < 3e-5 * max(1, abs(a))
        for k, v in ref_sd.items():
            assert torch.allclose(v, sd[k], atol=3e-5), k


@pytest.mark.parametrize("policy", ["block", "size"])
def test_full_shard_world1_aliased_matches_single_process(policy):
    """A shard group of one aliases each unit's gathered parameters / full gradient to its shard (no gather, scatter
    or free): same losses and parameters as plain AdamW, checkpoint consolidation included."""
    ref_losses, ref_sd = _reference()
    (losses, sd), = run_distributed(_worker, 1, "FULL_SHARD", policy)
    for a, b in zip(ref_losses, losses):
        assert abs(a - b) < 3e-5 * max(1, abs(a)), (ref_losses, losses)
    for k, v in ref_sd.items():
        assert torch.allclose(v, sd[k], atol=3e-5), k


def _worker_replicate_only(rank, world):
    """HYBRID with shard groups of one (aliased units) and gradients all-reduced over the replicate group."""
    from distributed_pytorch_hpc_amd.models.llama2 import TransformerBlock
    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ModuleWrapPolicy

    m = _model()
    singles = [dist.new_group([r]) for r in range(world)]
    f = FSDP(m, sharding_strategy="HYBRID_SHARD", auto_wrap_policy=ModuleWrapPolicy({TransformerBlock}),
             process_group=singles[rank], replicate_group=dist.new_group(list(range(world))))
    assert f.engine._alias
    opt = f.make_optimizer("adamw", lr=1e-2, weight_decay=0.1)
    losses = []
    for t in _batches():
        local = t.chunk(world, 0)[rank]
        loss = f(local[:, :-1], local[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        lt = loss.detach().clone()
        dist.all_reduce(lt)
        losses.append(lt.item() / world)
    return losses, f.full_state_dict(rank0_only=False)


def test_hybrid_shard_groups_of_one():
    ref_losses, ref_sd = _reference()
    for losses, sd in run_distributed(_worker_replicate_only, 2):
        for a, b in zip(ref_losses, losses):
            assert abs(a - b) < 3e-5 * max(1, abs(a))
        for k, v in ref_sd.items():
            assert torch.allclose(v, sd[k], atol=3e-5), k
