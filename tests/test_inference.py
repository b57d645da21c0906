"""Serving path (KV cache, incremental forward, Generator) on CPU: the reference ops are the oracles of the HIP
kernels (tests/test_decode_gpu.py), so the cached path must equal the full-sequence forward here."""
import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed


def _model(n_kv_heads=2, seed=0, vocab=97):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, Transformer

    torch.manual_seed(seed)
    return Transformer(ModelArgs(dim=64, n_layers=2, n_heads=4, n_kv_heads=n_kv_heads, vocab_size=vocab,
                                 multiple_of=32, max_seq_len=64)).float()


@pytest.mark.parametrize("n_kv_heads", [4, 2, 1])
def test_prefill_then_decode_matches_full_forward(n_kv_heads):
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _model(n_kv_heads)
    t = torch.randint(0, 97, (3, 14))
    full = m(t)
    c = KVCache(m, 3, 32)
    torch.testing.assert_close(m.forward_inference(t[:, :9], c), full[:, 8], atol=1e-5, rtol=1e-5)
    assert c.lengths == [9, 9, 9] and c.pos.tolist() == [9, 9, 9]
    for i in range(9, 14):
        torch.testing.assert_close(m.forward_inference(t[:, i:i + 1], c), full[:, i], atol=1e-5, rtol=1e-5)
    # a multi-token append after decode steps (chunked prefill / speculative verify) sees the whole prefix
    c.reset()
    m.forward_inference(t[:, :4], c)
    torch.testing.assert_close(m.forward_inference(t[:, 4:10], c, last_only=False), full[:, 4:10], atol=1e-5,
                               rtol=1e-5)


def test_ragged_prompts_through_cache_slots():
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _model()
    t = torch.randint(0, 97, (2, 12))
    full = m(t)
    c = KVCache(m, 2, 16)
    torch.testing.assert_close(m.forward_inference(t[:1, :5], c.slot(0)), full[0:1, 4], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.forward_inference(t[1:, :9], c.slot(1)), full[1:2, 8], atol=1e-5, rtol=1e-5)
    assert c.lengths == [5, 9] and c.length is None and c.attn_bound() == 10
    out = m.forward_inference(torch.stack([t[0, 5], t[1, 9]])[:, None], c)
    torch.testing.assert_close(out, torch.stack([full[0, 5], full[1, 9]]), atol=1e-5, rtol=1e-5)
    with pytest.raises(RuntimeError, match="same, host-known length"):
        m.forward_inference(t[:, :2], c)


def test_cache_capacity_is_enforced():
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _model()
    c = KVCache(m, 1, 8)
    m.forward_inference(torch.randint(0, 97, (1, 6)), c)
    with pytest.raises(ValueError, match="KV cache full"):
        m.forward_inference(torch.randint(0, 97, (1, 3)), c)
    with pytest.raises(ValueError, match="RoPE table"):
        KVCache(m, 1, 1000)


def test_generator_greedy_matches_naive_recompute():
    from distributed_pytorch_hpc_amd.inference import Generator

    m = _model()
    prompts = [[1, 2, 3, 4, 5], [7, 8, 9]]
    out = Generator(m, 2, 32).generate(prompts, 7)
    for p, o in zip(prompts, out):
        x = list(p)
        for _ in range(7):
            x.append(int(m(torch.tensor([x]))[0, -1].argmax()))
        assert o == x


def test_generator_sampling_eos_and_limits():
    from distributed_pytorch_hpc_amd.inference import Generator

    m = _model()
    g = Generator(m, 2, 16)
    a = g.generate([[3, 4], [5, 6]], 5, temperature=0.8, top_k=10, generator=torch.Generator().manual_seed(3))
    b = g.generate([[3, 4], [5, 6]], 5, temperature=0.8, top_k=10, generator=torch.Generator().manual_seed(3))
    assert a == b and all(len(r) == 7 for r in a)
    first = g.generate([[3, 4], [5, 6]], 1)
    stop = g.generate([[3, 4], [5, 6]], 6, eos_id=first[0][-1])
    assert stop[0] == first[0]                     # sequence 0 stops at its eos token
    with pytest.raises(ValueError, match="exceed the cache"):
        g.generate([[1] * 10, [2]], 8)


def _tp_generate_worker(rank, world):
    from distributed_pytorch_hpc_amd.inference import Generator
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama

    m = _model(vocab=96)
    parallelize_llama(m, dist.group.WORLD, sequence_parallel=False, loss_parallel=False)
    return Generator(m, 2, 32).generate([[1, 2, 3, 4, 5], [7, 8, 9, 10, 11]], 6)


def test_tensor_parallel_generation_matches_single_process():
    """TP=2 serving (heads and the KV cache sharded over ranks, gloo) emits the single-process greedy tokens."""
    from distributed_pytorch_hpc_amd.inference import Generator

    ref = Generator(_model(vocab=96), 2, 32).generate([[1, 2, 3, 4, 5], [7, 8, 9, 10, 11]], 6)
    for out in run_distributed(_tp_generate_worker, 2):
        assert out == ref


def test_continuous_batching_matches_one_request_at_a_time():
    """5 requests of different lengths on 2 cache slots: every output equals that request generated alone."""
    from distributed_pytorch_hpc_amd.inference import ContinuousBatcher, Generator

    m = _model()
    reqs = [([1, 2, 3], 5), ([4, 5, 6, 7, 8, 9], 3), ([10], 6), ([11, 12], 1), ([13, 14, 15, 16], 4)]
    cb = ContinuousBatcher(Generator(m, 2, 16))
    handles = [cb.submit(p, n) for p, n in reqs]
    done = cb.run()
    assert len(done) == len(reqs) and all(h.done for h in handles) and cb.active == 0
    solo = Generator(m, 1, 16)
    for h, (p, n) in zip(handles, reqs):
        assert h.prompt + h.output == solo.generate([p], n)[0]


def test_fp8_kv_cache_tracks_the_full_forward():
    """OCP e4m3 cache entries (x / kv_scale): prefill + decode logits stay close to the exact full forward."""
    from distributed_pytorch_hpc_amd.models.llama2 import KVCache

    m = _model()
    t = torch.randint(0, 97, (2, 16))
    full = m(t)
    c = KVCache(m, 2, 32, dtype=torch.float8_e4m3fn, kv_scale=0.5)
    assert c.fp8 and c.k.dtype == torch.float8_e4m3fn
    got = [m.forward_inference(t[:, :10], c)]
    got += [m.forward_inference(t[:, i:i + 1], c) for i in range(10, 13)]
    got.append(m.forward_inference(t[:, 13:16], c, last_only=False)[:, -1])   # chunked append over an fp8 prefix
    got = torch.stack(got, 1)
    ref = torch.stack([full[:, 9], full[:, 10], full[:, 11], full[:, 12], full[:, 15]], 1)
    assert (got - ref).norm() / ref.norm() < 0.05
