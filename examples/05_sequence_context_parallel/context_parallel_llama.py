#!/usr/bin/env python3
"""Long-context Llama training with context parallelism: DeepSpeed-Ulysses or ring attention over a cp group.

Reference: documented only (docs/guide/08_sequence_parallel.md:41-142 -- Ulysses all-to-all pseudocode, ring
attention with per-step K/V isend/irecv and an online-softmax merge; scripts advertised in README.md:58,69 do
not exist: reference gap X1).

Each rank holds a contiguous S/cp slice of every sequence (RoPE uses global positions).  ``ulysses``: all-to-all
q/k/v from sequence-sharded to head-sharded, full-length flash attention on H/cp heads, all-to-all back
(needs heads % cp == 0).  ``ring``: K/V blocks (+ their dK/dV accumulators in backward) rotate around the cp
ring while the flash kernel merges partial (o, lse) results.  Gradients are averaged over all dp x cp ranks by
the bucketed engine.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/05_sequence_context_parallel/context_parallel_llama.py \
        --mode ring --cp 8 --model llama2-1b --seq-len 32768
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import Mesh  # noqa: E402
from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.context_parallel import apply_context_parallel, shard_sequence  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.utils.metrics import sync  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--mode", choices=["ulysses", "ring"], default="ulysses")
    ap.add_argument("--cp", type=int, default=None, help="context-parallel degree (default: world)")
    ap.add_argument("--layout", choices=["auto", "contiguous", "zigzag"], default="auto",
                    help="sequence sharding; auto = zigzag (load-balanced causal) for ring, contiguous for Ulysses")
    ap.add_argument("--model", default="toy")
    ap.add_argument("--n-layers", type=int, default=None)
    ap.add_argument("--seq-len", type=int, default=1024, help="GLOBAL sequence length")
    ap.add_argument("--batch", type=int, default=1, help="sequences per dp replica")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--lr", type=float, default=3e-4)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    cp = args.cp or world
    assert world % cp == 0 and args.seq_len % cp == 0
    mesh = Mesh((world // cp, cp), ("dp", "cp"))
    cp_rank, dp_rank = mesh.local_rank("cp"), mesh.local_rank("dp")

    over = {"max_seq_len": max(args.seq_len, 512)}
    if args.n_layers:
        over["n_layers"] = args.n_layers
    margs = get_preset(args.model, **over)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model = build_llama(margs, device=dev, dtype=dtype, seed=args.seed)
    layout = args.layout if args.layout != "auto" else ("zigzag" if args.mode == "ring" else "contiguous")
    apply_context_parallel(model, mesh.group("cp"), args.mode, layout=layout)
    engine = DataParallelEngine(model, None, shard=world > 1 and dev.type == "cuda")
    engine.configure_optimizer(OptimConfig("adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    s_loc = args.seq_len // cp
    g = torch.Generator(device=dev).manual_seed(args.seed + dp_rank)
    times = []
    for step in range(args.warmup + args.steps):
        t = torch.randint(0, margs.vocab_size, (args.batch, args.seq_len + 1), device=dev, generator=g)
        x = shard_sequence(t[:, :-1], mesh.group("cp"), layout)
        y = shard_sequence(t[:, 1:], mesh.group("cp"), layout)
        sync()
        t0 = time.perf_counter()
        loss = model(x, y)
        loss.backward()
        engine.step()
        engine.zero_grad()
        sync()
        if step >= args.warmup:
            times.append(time.perf_counter() - t0)
        lt = loss.detach().float().clone()
        if world > 1:
            dist.all_reduce(lt)
        if rank == 0:
            print(f"step {step}: loss {lt.item() / world:.4f}", flush=True)
    engine.synchronize()
    step_t = sum(times) / len(times)
    tps = args.batch * args.seq_len * (world // cp) / step_t
    summary = {"example": "context_parallel_llama", "mode": args.mode, "layout": layout, "cp": cp, "dp": world // cp,
               "model": args.model, "seq_len": args.seq_len, "ms_per_step": 1000 * step_t,
               "tokens_per_sec": tps, "final_loss": lt.item() / world}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
