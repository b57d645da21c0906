"""Checkpoint/resume: consolidated round trip, sharded save at dp=2 -> resume at dp=2 and at dp=1 (reshard)."""
import os

import torch
import torch.distributed as dist

from dist_utils import run_distributed

PRESET = dict(dim=64, n_layers=2, n_heads=4, vocab_size=128, max_seq_len=64, multiple_of=32)


def _setup(shard, bucket_mb=0.02):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=5)
    eng = DataParallelEngine(m, shard=shard, bucket_cap_mb=bucket_mb)
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


def _resume_single(root, bucket_mb=0.02):
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    m, eng = _setup(False, bucket_mb)
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


def _slices_save_load(rank, world, root):
    """World 4 = 2 model-parallel slices (ranks {0,1} and {2,3}, a different model each, as TP shards would be) x
    dp 2.  Only dp-rank 0 of a slice writes its model; every rank must get ITS slice back."""
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
    sl = rank // 2
    dpg = groups[sl]

    def setup(seed):
        m = build_llama(ModelArgs(**PRESET), device="cpu", dtype=torch.float32, seed=seed)
        # parameters come back through the restored fp32 masters either way; a buffer only through the model file
        m.register_buffer("slice_tag", torch.full((4,), float(seed)))
        eng = DataParallelEngine(m, process_group=dpg, shard=True, bucket_cap_mb=0.02)
        eng.configure_optimizer(OptimConfig(lr=1e-2))
        return m, eng

    m, eng = setup(100 + sl)
    g = torch.Generator().manual_seed(20 + sl)
    for _ in range(2):
        t = torch.randint(0, 128, (4, 17), generator=g).chunk(2, 0)[dist.get_rank(dpg)]
        m(t[:, :-1], t[:, 1:]).backward()
        eng.step()
        eng.zero_grad()
    eng.synchronize()
    saved = {k: v.clone() for k, v in m.state_dict().items()}
    ShardedCheckpointer(root, m, eng).save(2)
    m2, eng2 = setup(999)
    assert ShardedCheckpointer(root, m2, eng2).load() == 2
    for k, v in m2.state_dict().items():
        assert torch.equal(v, saved[k]), (rank, k)
    assert torch.equal(eng2.master, eng.master) and eng2.step_count == 2
    return sl


def test_sharded_model_parallel_slices_resume(tmp_path):
    assert run_distributed(_slices_save_load, 4, str(tmp_path)) == [0, 0, 1, 1]


def test_sharded_resume_reshard_to_one_rank(tmp_path):
    # save at dp=2 (sharded optimizer), resume on a single rank
    run_distributed(_save_then_resume, 2, str(tmp_path), True)
    ref = run_distributed(_uninterrupted, 2)[0]
    got = _resume_single(str(tmp_path))
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-5), k


def test_sharded_resume_reshard_other_bucket_partition(tmp_path):
    """Resume at dp=1 with another bucket size (the 'calibrate' / 'auto' sizes depend on the world): the state is
    re-cut from the saved group sizes, and the fp32 master AND the AdamW moments come back."""
    run_distributed(_save_then_resume, 2, str(tmp_path), True)
    ref = run_distributed(_uninterrupted, 2)[0]
    got = _resume_single(str(tmp_path), bucket_mb=0.05)
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-5), k


def test_reshard_without_group_sizes_refuses_other_partition(tmp_path):
    """An older checkpoint (no recorded group sizes) whose partition differs must raise, not silently skip."""
    import glob

    import pytest

    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    run_distributed(_save_then_resume, 2, str(tmp_path), True)
    for f in glob.glob(os.path.join(str(tmp_path), "**", "rank*.pt"), recursive=True):
        st = torch.load(f, map_location="cpu", weights_only=True)
        st["optim"].pop("group_real", None)
        torch.save(st, f)
    m, eng = _setup(False, bucket_mb=0.05)
    with pytest.raises(ValueError, match="bucket partition"):   # caught by the master-vs-weights check
        ShardedCheckpointer(str(tmp_path), m, eng).load()


# ------------------------------------------------------------------------------------------------ FSDP / ZeRO engines
# FULL_SHARD releases the module's parameter storage between uses (parallel/fsdp.py ZeRO3Engine): checkpoints must
# gather the full state and load it back into the shards, for the consolidated and the sharded format, at the same
# and at another world size, and across strategies.
def _fsdp_setup(strategy="FULL_SHARD"):
    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, size_based_auto_wrap_policy

    torch.manual_seed(3)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 32), torch.nn.ReLU(),
                            torch.nn.Linear(32, 8))
    f = FSDP(m, sharding_strategy=strategy, auto_wrap_policy=size_based_auto_wrap_policy(1))
    return f, f.make_optimizer("adamw", lr=1e-2, weight_decay=0.1)


def _fsdp_batches(n):
    g = torch.Generator().manual_seed(11)
    return [(torch.randn(8, 16, generator=g), torch.randn(8, 8, generator=g)) for _ in range(n)]


def _fsdp_train(f, opt, batches, rank, world):
    for x, y in batches:
        opt.zero_grad()
        torch.nn.functional.mse_loss(f(x.chunk(world)[rank]), y.chunk(world)[rank]).backward()
        opt.step()
    f.engine.synchronize()


def _fsdp_uninterrupted(rank, world, strategy):
    f, opt = _fsdp_setup(strategy)
    _fsdp_train(f, opt, _fsdp_batches(4), rank, world)
    return f.full_state_dict(rank0_only=False)


def _fsdp_consolidated_save(rank, world, path, strategy):
    from distributed_pytorch_hpc_amd.utils.checkpointing import save_checkpoint

    f, opt = _fsdp_setup(strategy)
    _fsdp_train(f, opt, _fsdp_batches(4)[:2], rank, world)
    save_checkpoint(f, opt, 2, path)
    return {}


def _fsdp_consolidated_resume(rank, world, path, strategy):
    from distributed_pytorch_hpc_amd.utils.checkpointing import load_checkpoint

    f, opt = _fsdp_setup(strategy)
    assert load_checkpoint(f, opt, path) == 2
    assert opt.engine.step_count == 2
    _fsdp_train(f, opt, _fsdp_batches(4)[2:], rank, world)
    return f.full_state_dict(rank0_only=False)


def _fsdp_sharded_save(rank, world, root):
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    f, opt = _fsdp_setup()
    _fsdp_train(f, opt, _fsdp_batches(4)[:2], rank, world)
    ShardedCheckpointer(root, f).save(2)
    return {}


def _fsdp_sharded_resume(rank, world, root):
    from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer

    f, opt = _fsdp_setup()
    assert ShardedCheckpointer(root, f).load() == 2
    _fsdp_train(f, opt, _fsdp_batches(4)[2:], rank, world)
    return f.full_state_dict(rank0_only=False)


def _close(ref, got, atol=1e-5):
    assert ref.keys() == got.keys()
    for k in ref:
        assert ref[k].numel() > 0 and torch.allclose(ref[k], got[k], atol=atol), k


def test_fsdp_full_shard_consolidated_single_rank(tmp_path):
    """World 1 in-process: the saved file holds real (non-empty) tensors and loads into a fresh FSDP model."""
    import torch.distributed as d

    p = str(tmp_path / "ck.pt")
    d.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        ref = _fsdp_uninterrupted(0, 1, "FULL_SHARD")
        _fsdp_consolidated_save(0, 1, p, "FULL_SHARD")
        sd = torch.load(p, weights_only=True)
        assert all(v.numel() > 0 for v in sd["model_state_dict"].values())
        assert sd["optimizer_state_dict"]["format"] == "full"
        got = _fsdp_consolidated_resume(0, 1, p, "FULL_SHARD")
    finally:
        d.destroy_process_group()
    _close(ref, got)


def test_fsdp_full_shard_consolidated_two_ranks_resume_on_one(tmp_path):
    p = str(tmp_path / "ck.pt")
    ref = run_distributed(_fsdp_uninterrupted, 2, "FULL_SHARD")[0]
    run_distributed(_fsdp_consolidated_save, 2, p, "FULL_SHARD")
    got2 = run_distributed(_fsdp_consolidated_resume, 2, p, "FULL_SHARD")[0]
    _close(ref, got2)
    # the same file into another strategy (DDP-style NO_SHARD) and world size
    got1 = run_distributed(_fsdp_consolidated_resume, 1, p, "NO_SHARD")[0]
    _close(ref, got1)


def test_fsdp_full_shard_sharded_checkpointer_reshard(tmp_path):
    root = str(tmp_path / "ck")
    ref = run_distributed(_fsdp_uninterrupted, 2, "FULL_SHARD")[0]
    run_distributed(_fsdp_sharded_save, 2, root)
    _close(ref, run_distributed(_fsdp_sharded_resume, 2, root)[0])
    _close(ref, run_distributed(_fsdp_sharded_resume, 1, root)[0])


def test_fsdp_full_shard_load_rejects_wrong_shape():
    """A same-numel tensor of another shape (a transposed weight) must not load silently in scrambled order."""
    import pytest

    f, _ = _fsdp_setup()
    sd = f.full_state_dict(rank0_only=False)
    sd["2.weight"] = sd["2.weight"].t().contiguous()        # 32 x 32: same numel, transposed
    sd["0.weight"] = sd["0.weight"].reshape(16, 32)          # 32 x 16 -> 16 x 32
    with pytest.raises(ValueError, match=r"size mismatch for 0\.weight"):
        f.load_state_dict(sd)
