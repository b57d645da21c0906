"""Checkpoint/resume: consolidated round trip, sharded save at dp=2 -> resume at dp=2 and at dp=1 (reshard)."""
import os

import torch
import torch.distributed as dist

from dist_utils import run_distributed

PRESET = dict(dim=64, n_layers=2, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)


def _setup(shard):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=5)
    eng = DataParallelEngine(m, shard=shard, bucket_cap_mb=0.02)
    eng.configure_optimizer(OptimConfig(lr=1e-2, weight_decay=0.1))
    return m, eng


def _batches(n):
    g = torch.Generator().manual_seed(8)
    return [torch.randint(0, 128, (4, 17), generator=g) for _ in range(n)]


def _train(m, eng, batches, rank, world):
    for t in batches:
        local = t.chunk(world, 0)[rank]
        loss = m(local[:, :-1], local[:, 1:])
        loss.backward()
        eng.step()
        eng.zero_grad()
    eng.synchronize()


def _uninterrupted(rank, world):
    m, eng = _setup(world > 1)
    _train(m, eng, _batches(4), rank, world)
    return {k: v.clone() for k, v in m.state_dict().items()}


def _save_then_resume(rank, world, root, resume_world_same):
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    m, eng = _setup(world > 1)
    b = _batches(4)
    _train(m, eng, b[:2], rank, world)
    ck = ShardedCheckpointer(root, m, eng)
    ck.save(2)
    # fresh model/engine, resume, finish
    m2, eng2 = _setup(world > 1)
    step = ShardedCheckpointer(root, m2, eng2).load()
    assert step == 2
    _train(m2, eng2, b[2:], rank, world)
    return {k: v.clone() for k, v in m2.state_dict().items()}


def _resume_single(root):
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    m, eng = _setup(False)
    step = ShardedCheckpointer(root, m, eng).load()
    assert step == 2
    _train(m, eng, _batches(4)[2:], 0, 1)
    return {k: v.clone() for k, v in m.state_dict().items()}


def test_consolidated_roundtrip(tmp_path):
    from distributed_pytorch_hpc_amd.train.optim import FusedAdamW
    from distributed_pytorch_hpc_amd.utils.checkpointing import load_checkpoint, save_checkpoint

    lin = torch.nn.Linear(8, 4)
    opt = FusedAdamW(lin.parameters(), lr=0.1)
    lin(torch.randn(3, 8)).sum().backward()
    opt.step()
    p = str(tmp_path / "ck.pt")
    save_checkpoint(lin, opt, 7, p)
    lin2 = torch.nn.Linear(8, 4)
    opt2 = FusedAdamW(lin2.parameters(), lr=0.1)
    assert load_checkpoint(lin2, opt2, p) == 7
    for a, b in zip(lin.parameters(), lin2.parameters()):
        assert torch.equal(a, b)
    assert opt2.flat_states()[0].step == 1


def test_sharded_resume_same_world(tmp_path):
    ref = run_distributed(_uninterrupted, 2)[0]
    got = run_distributed(_save_then_resume, 2, str(tmp_path), True)[0]
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-6), k


def test_sharded_resume_reshard_to_one_rank(tmp_path):
    # save at dp=2 (sharded optimizer), resume on a single rank
    run_distributed(_save_then_resume, 2, str(tmp_path), True)
    ref = run_distributed(_uninterrupted, 2)[0]
    got = _resume_single(str(tmp_path))
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-5), k
