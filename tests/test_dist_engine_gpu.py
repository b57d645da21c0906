"""Two ranks sharing one MI355X (gloo process group, bf16 Llama with the HIP kernels): the sharded engine
(reduce-scatter, 1/N AdamW on the HIP optimizer kernel, asynchronous all-gather waited on in the next forward) must
reproduce the replicated DDP engine step for step.  This is the N > 1 path `bench.py` takes on 2..8 GPUs, run here
on GPU tensors; RCCL itself needs one GPU per rank and is covered by the round-end multi-GPU bench.
"""
import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed

pytestmark = pytest.mark.gpu

STEPS = 3
PRESET = dict(dim=256, n_layers=2, n_heads=4, vocab_size=512, max_seq_len=256, multiple_of=64)


def _run(rank, world, shard):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    _lib.require()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = build_llama(ModelArgs(**PRESET), device=dev, dtype=torch.bfloat16, seed=11)
    eng = DataParallelEngine(m, shard=shard, bucket_cap_mb=0.25)
    eng.configure_optimizer(OptimConfig(lr=1e-3, weight_decay=0.1))
    g = torch.Generator().manual_seed(5)
    losses = []
    for _ in range(STEPS):
        t = torch.randint(0, PRESET["vocab_size"], (2 * world, 129), generator=g).chunk(world, 0)[rank].to(dev)
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        eng.step()
        eng.zero_grad()
        lt = loss.detach().float().clone()
        dist.all_reduce(lt)
        losses.append(lt.item() / world)
    eng.synchronize()
    torch.cuda.synchronize()
    return losses, {k: v.detach().float().cpu() for k, v in m.state_dict().items()}


def _worker(rank, world):
    return _run(rank, world, False), _run(rank, world, True)


def test_sharded_engine_matches_ddp_two_ranks_one_gpu():
    outs = run_distributed(_worker, 2, timeout=110.0)
    (ddp_l, ddp_sd), _ = outs[0]
    for (l_ddp, sd_ddp), (l_sh, sd_sh) in outs:
        assert l_ddp == pytest.approx(ddp_l, rel=1e-6)           # DDP replicas agree
        assert l_sh == pytest.approx(l_ddp, rel=2e-3), (l_sh, l_ddp)
        for k, v in sd_ddp.items():
            assert torch.equal(v, ddp_sd[k]), k                      # replicas bitwise identical
            torch.testing.assert_close(sd_sh[k], v, atol=2e-3, rtol=2e-2, msg=k)
    assert ddp_l[-1] < ddp_l[0]
