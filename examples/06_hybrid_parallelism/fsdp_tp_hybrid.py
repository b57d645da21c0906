#!/usr/bin/env python3
"""2-D hybrid parallelism for Llama-2: sharded data parallel (dp) x tensor + sequence parallel (tp).

Reference: scripts/06_hybrid_parallelism/01_fsdp_tp_hybrid.py and fsdp_tp/fsdp_tp_example.py (Llama toy dim 256,
2 layers, 16 heads, vocab 32000; ``init_device_mesh((dp, tp), ("dp", "tp"))`` with tp = 4 hard-coded; the
TorchTitan TP+SP plan; ``fully_shard(model, mesh=dp_mesh)`` on the ROOT only; AdamW lr 3e-3 foreach; inputs
seeded with ``i + dp_rank``; loss = output.sum(); "2D iter i complete").

MI355X version: real ``--tp`` / ``--dp`` flags (reference defect X10), TP applied first (column/row shards of
the fused QKV / W1||W3 projections, sequence-parallel norms, reduce-scatter after wo / w2), then the bucketed
ZeRO engine shards gradients + optimizer state over dp (reference X8: root-only FSDP2), ``zero_grad`` every
step (X7), vocab-parallel cross-entropy on sharded logits (no [B, S, V] all-gather).  ``--loss sum`` reproduces
the reference's output.sum() objective.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/06_hybrid_parallelism/fsdp_tp_hybrid.py --tp 4
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/06_hybrid_parallelism/fsdp_tp_hybrid.py \
        --model llama2-7b --tp 8 --batch 8 --seq-len 4096 --iters 10
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D  # noqa: E402
from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, MixedPrecision, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.utils.metrics import sync  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--tp", type=int, default=None, help="tensor-parallel degree (default: min(4, world))")
    ap.add_argument("--dp", type=int, default=None, help="data-parallel degree (default: world // tp)")
    ap.add_argument("--model", default="toy")
    ap.add_argument("--n-layers", type=int, default=None)
    ap.add_argument("--batch", type=int, default=8, help="sequences per dp replica")
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--loss", choices=["ce", "sum"], default="ce")
    ap.add_argument("--no-sp", action="store_true", help="disable sequence parallelism")
    ap.add_argument("--no-loss-parallel", action="store_true")
    ap.add_argument("--async-tp", type=int, default=0,
                    help="k > 0: pipeline the SP all-gathers / reduce-scatters against the projection GEMMs in k "
                         "micro-collectives (parallel/async_tp.py)")
    ap.add_argument("--no-shard", action="store_true", help="replicated optimizer state over dp (plain DDP)")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    tp = args.tp or min(4, world)
    dp = args.dp or world // tp
    assert dp * tp == world, f"dp {dp} x tp {tp} != world {world}"
    mesh = DeviceMesh2D(dp, tp)

    over = {"max_seq_len": max(args.seq_len, 512)}
    if args.n_layers:
        over["n_layers"] = args.n_layers
    margs = get_preset(args.model, **over)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model = build_llama(margs, device=dev, dtype=dtype, seed=args.seed)
    n_params = sum(p.numel() for p in model.parameters())
    parallelize_llama(model, mesh.tp_group, sequence_parallel=not args.no_sp,
                      loss_parallel=not args.no_loss_parallel and args.loss == "ce",
                      async_tp=0 if args.no_sp else args.async_tp)
    engine = DataParallelEngine(model, mesh.dp_group, shard=not args.no_shard and dp > 1,
                                mixed_precision=MixedPrecision(reduce_dtype=dtype))
    engine.configure_optimizer(OptimConfig("adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    if rank == 0:
        print(f"[hybrid] {args.model}: {n_params:,} params | mesh dp={dp} x tp={tp} | sp={not args.no_sp}",
              flush=True)
    times, losses = [], []
    for i in range(args.iters):
        g = torch.Generator(device=dev).manual_seed(i + mesh.dp_rank)   # TP peers share the batch
        t = torch.randint(0, margs.vocab_size, (args.batch, args.seq_len + 1), device=dev, generator=g)
        sync()
        t0 = time.perf_counter()
        if args.loss == "sum":
            loss = model(t[:, :-1]).sum()
        else:
            loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        engine.step()
        engine.zero_grad()
        sync()
        times.append(time.perf_counter() - t0)
        lt = loss.detach().float().clone()
        if dp > 1:
            dist.all_reduce(lt, group=mesh.dp_group)
        losses.append(lt.item() / dp)
        if rank == 0:
            print(f"2D iter {i} complete | loss {losses[-1]:.4f} | {1000 * times[-1]:.1f} ms", flush=True)
    engine.synchronize()
    steady = times[1:] if len(times) > 1 else times
    step_t = sum(steady) / len(steady)
    summary = {"example": "fsdp_tp_hybrid", "model": args.model, "dp": dp, "tp": tp, "params": n_params,
               "losses": losses, "ms_per_step": 1000 * step_t,
               "tokens_per_sec": args.batch * args.seq_len * dp / step_t}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
