#!/usr/bin/env python3
"""3-D parallelism for Llama-2: pipeline (pp) x data (dp) x tensor+sequence (tp) on one process mesh.

Reference: documented only (docs/guide/09_hybrid_parallelism.md:141-159 and scripts/06_hybrid_parallelism/
README.md:104-113 describe TP+PP+FSDP(+SP) "3-D/4-D" layouts; no script exists).

Layout: ``Mesh((pp, dp, tp), ("pp", "dp", "tp"))`` with tp fastest-varying.  TP (+SP, vocab-parallel loss) is
applied to the whole model, the model is then cut into ``pp`` contiguous layer ranges (parallel/pipeline.py
LlamaStage), each stage trains with the 1F1B schedule over its pp group (activations stay sequence-sharded
between stages), and the stage's gradients are reduced (sharded optimizer state when dp > 1) over its dp group,
deferred to the last micro-batch.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/06_hybrid_parallelism/three_d_parallel.py \
        --pp 2 --dp 2 --tp 2
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import Mesh  # noqa: E402
from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, make_lm_loss, split_llama  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.utils.metrics import sync  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--pp", type=int, default=2)
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--tp", type=int, default=None, help="default world // (pp * dp)")
    ap.add_argument("--model", default="toy")
    ap.add_argument("--n-layers", type=int, default=None)
    ap.add_argument("--batch", type=int, default=8, help="sequences per dp replica")
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--microbatches", type=int, default=4)
    ap.add_argument("--schedule", choices=["1f1b", "gpipe"], default="1f1b")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lr", type=float, default=1e-3)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    tp = args.tp or world // (args.pp * args.dp)
    assert args.pp * args.dp * tp == world, "pp * dp * tp must equal the world size"
    mesh = Mesh((args.pp, args.dp, tp), ("pp", "dp", "tp"))
    stage, dp_rank = mesh.local_rank("pp"), mesh.local_rank("dp")

    over = {"max_seq_len": max(args.seq_len, 512)}
    if args.n_layers:
        over["n_layers"] = args.n_layers
    margs = get_preset(args.model, **over)
    assert margs.n_layers >= args.pp
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model = build_llama(margs, device=dev, dtype=dtype, seed=args.seed)
    tp_group = mesh.group("tp")
    if tp > 1:
        parallelize_llama(model, tp_group, sequence_parallel=True, loss_parallel=True)
    stage_mod = split_llama(model, args.pp, stage)
    del model
    engine = DataParallelEngine(stage_mod, mesh.group("dp"), shard=args.dp > 1)
    engine.configure_optimizer(OptimConfig("adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    sched = PipelineSchedule(stage_mod, stage, args.pp, args.microbatches,
                             loss_fn=make_lm_loss(tp_group if tp > 1 else None, loss_parallel=tp > 1),
                             group=mesh.group("pp"), schedule=args.schedule, device=dev,
                             dp_engine=engine)
    times, losses = [], []
    last = stage == args.pp - 1
    for i in range(args.iters):
        g = torch.Generator(device=dev).manual_seed(1000 * i + dp_rank)
        t = torch.randint(0, margs.vocab_size, (args.batch, args.seq_len + 1), device=dev, generator=g)
        sync()
        t0 = time.perf_counter()
        mb_losses = sched.step(inputs=t[:, :-1] if stage == 0 else None, target=t[:, 1:] if last else None)
        engine.step()
        engine.zero_grad()
        sync()
        times.append(time.perf_counter() - t0)
        lt = torch.stack(mb_losses).mean().float() if mb_losses else torch.zeros((), device=dev)
        if world > 1:
            dist.all_reduce(lt)   # only last-stage ranks contribute (tp * dp of them)
        losses.append(lt.item() / (tp * args.dp))
        if rank == 0:
            print(f"3D iter {i}: loss {losses[-1]:.4f} | {1000 * times[-1]:.1f} ms", flush=True)
    engine.synchronize()
    steady = times[1:] if len(times) > 1 else times
    step_t = sum(steady) / len(steady)
    summary = {"example": "three_d_parallel", "pp": args.pp, "dp": args.dp, "tp": tp, "losses": losses,
               "ms_per_step": 1000 * step_t, "tokens_per_sec": args.batch * args.seq_len * args.dp / step_t,
               "bubble_fraction": sched.bubble}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
