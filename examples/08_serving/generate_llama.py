#!/usr/bin/env python3
"""Llama text generation with a KV cache: prefill + HIP-graph decode, optionally tensor-parallel across ranks.

Reference: none -- the reference trains only (fsdp_tp/llama2_model.py has no cache or generate loop); this is the
serving side of the same model on MI355X (models/llama2.py KVCache, inference/generator.py, csrc/decode.hip).

One rank: the whole model on one GPU (a 7B bf16 model is 13.5 GB of the 288 GB; the rest holds KV caches: 0.5 MiB per
token and sequence at 7B).  N ranks: Megatron tensor parallelism (heads, FFN and the KV cache split over the ranks,
one all-reduce after wo and w2 per layer over RCCL/xGMI).  Weights are random unless ``--checkpoint`` names a model
state dict saved by this framework (loaded with ``torch.load(weights_only=True)``); prompts are synthetic ids.

    python examples/08_serving/generate_llama.py --model llama2-7b --batch 8 --prompt-len 1024 --max-new 128
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/08_serving/generate_llama.py --model llama2-7b
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.inference import Generator  # noqa: E402
from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--model", default="tiny")
    ap.add_argument("--n-layers", type=int, default=None)
    ap.add_argument("--checkpoint", default=None, help="model state dict (torch.save of model.state_dict())")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--max-new", type=int, default=32)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-k", type=int, default=None)
    ap.add_argument("--no-graphs", action="store_true", help="eager decode steps (default: HIP graphs on one GPU)")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    over = {"max_seq_len": max(args.prompt_len + args.max_new, 64)}
    if args.n_layers:
        over["n_layers"] = args.n_layers
    margs = get_preset(args.model, **over)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model = build_llama(margs, device=dev, dtype=dtype, seed=args.seed)
    if args.checkpoint:
        model.load_state_dict(torch.load(args.checkpoint, map_location=dev, weights_only=True))
    if world > 1:
        parallelize_llama(model, dist.group.WORLD, sequence_parallel=False, loss_parallel=False)
    model.eval()
    g = torch.Generator().manual_seed(args.seed)   # the same prompts on every rank
    prompts = torch.randint(0, margs.vocab_size, (args.batch, args.prompt_len), generator=g)

    graphs = dev.type == "cuda" and world == 1 and not args.no_graphs
    gen = Generator(model, args.batch, args.prompt_len + args.max_new, graphs=graphs)
    gen.generate(prompts, 2)   # warm-up: library set-up (and the graph capture on the first decode steps)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    gen.reset()
    logits = gen.prefill(prompts)
    sync()
    t_prefill = time.perf_counter() - t0
    samp = torch.Generator(device=dev).manual_seed(args.seed) if args.temperature > 0 else None
    tok = gen.sample(logits, args.temperature, args.top_k, samp)
    out = [tok]
    t1 = time.perf_counter()
    for _ in range(args.max_new - 1):
        tok = gen.sample(gen.decode(tok), args.temperature, args.top_k, samp)
        out.append(tok)
    sync()
    t_decode = time.perf_counter() - t1
    new = torch.stack(out, 1).cpu()
    steps = max(args.max_new - 1, 1)
    summary = {"example": "generate_llama", "model": args.model, "tp": world, "batch": args.batch,
               "prompt_len": args.prompt_len, "new_tokens": args.max_new, "graphs": graphs,
               "prefill_tokens_per_sec": args.batch * args.prompt_len / t_prefill,
               "decode_ms_per_step": 1000 * t_decode / steps,
               "decode_tokens_per_sec": args.batch * steps / t_decode,
               "first_sequence_new_ids": new[0, :16].tolist()}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
