"""Activation checkpointing: identical loss and gradients with and without recompute (CPU)."""
import torch

from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama, get_preset
from distributed_pytorch_hpc_amd.parallel.activation_checkpoint import (CheckpointWrapper, apply_llama_checkpointing,
                                                                        plan_llama_checkpointing)
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

ARGS = ModelArgs(dim=64, n_layers=4, n_heads=4, vocab_size=97, max_seq_len=64)


def _grads(every):
    m = build_llama(ARGS, device="cpu", dtype=torch.float32, seed=5)
    n = apply_llama_checkpointing(m, every) if every else 0
    eng = DataParallelEngine(m)
    eng.configure_optimizer(OptimConfig("sgd", lr=0.0))
    t = torch.randint(0, 97, (2, 33), generator=torch.Generator().manual_seed(0))
    loss = m(t[:, :-1], t[:, 1:])
    loss.backward()
    return n, loss.item(), eng.flat_grad.clone()


def test_checkpointed_llama_matches_plain():
    _, l0, g0 = _grads(0)
    for every in (1, 2):
        n, l1, g1 = _grads(every)
        assert n == (4 if every == 1 else 2)
        assert abs(l0 - l1) < 1e-6
        torch.testing.assert_close(g1, g0, rtol=1e-5, atol=1e-6)


def test_wrapper_forwards_attributes():
    m = build_llama(ARGS, device="cpu", dtype=torch.float32, seed=5)
    apply_llama_checkpointing(m, 1)
    assert isinstance(m.layers[0], CheckpointWrapper)
    assert m.layers[0].attention is m.layers[0].module.attention


def test_plan_fits_7b_without_checkpointing_at_bench_config():
    args = get_preset("llama2-7b")
    assert plan_llama_checkpointing(args, 8, 4096, static_gb=108) == 0     # bench.py config: no recompute
    assert plan_llama_checkpointing(args, 8, 32768, static_gb=108) >= 1    # 8 x 32k tokens needs recompute
