#!/usr/bin/env python3
"""FSDP UNet on ERA5-shaped fields + consolidated FULL_STATE_DICT checkpoint from rank 0.

Reference: scripts/02_fully_sharded_fsdp/multinode_fsdp_unet.py:134-316 (SimpleUNet, size-based wrap policy
1e5 params, FULL_SHARD, fp32, AdamW, latitude-weighted MSE, samples/s; FULL_STATE_DICT with
``offload_to_cpu=True, rank0_only=True`` saved at the end, L285-298).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/02_fully_sharded_fsdp/fsdp_unet.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from distributed_pytorch_hpc_amd.data import DeviceBatches  # noqa: E402
from distributed_pytorch_hpc_amd.models import SimpleUNet  # noqa: E402
from distributed_pytorch_hpc_amd.ops import latitude_weighted_mse  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import MixedPrecision  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ShardingStrategy, size_based_auto_wrap_policy  # noqa: E402
from distributed_pytorch_hpc_amd.train import Trainer  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--steps-per-epoch", type=int, default=20)
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--channels", type=int, default=65)
    ap.add_argument("--lat", type=int, default=181)
    ap.add_argument("--lon", type=int, default=360)
    ap.add_argument("--base-dim", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--weight-decay", type=float, default=1e-5)
    ap.add_argument("--sharding", default="FULL_SHARD", choices=[s.value for s in ShardingStrategy])
    ap.add_argument("--bf16", action="store_true", help="MixedPrecision(param=bf16, reduce=bf16)")
    ap.add_argument("--checkpoint", default=None, help="FULL_STATE_DICT output path (rank 0)")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    model = SimpleUNet(args.channels, args.channels, args.base_dim).to(dev)
    n_params = sum(p.numel() for p in model.parameters())
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if args.bf16 else None
    fsdp = FSDP(model, sharding_strategy=args.sharding, mixed_precision=mp,
                auto_wrap_policy=size_based_auto_wrap_policy(int(1e5)))
    opt = fsdp.make_optimizer("adamw", lr=args.lr, weight_decay=args.weight_decay)
    data = DeviceBatches("era5", args.batch_size, dev, seed=args.seed, rank=rank, channels=args.channels,
                         lat=args.lat, lon=args.lon, dtype=torch.bfloat16 if args.bf16 else torch.float32)
    trainer = Trainer(fsdp, opt, data, lambda o, t: latitude_weighted_mse(o.float(), t.float()), dev,
                      max_steps_per_epoch=args.steps_per_epoch, log_every=max(args.steps_per_epoch // 4, 1),
                      metrics_file=args.metrics_file,
                      cuda_graph=args.cuda_graph)
    summary = trainer.train(args.epochs)
    if args.checkpoint:
        sd = fsdp.full_state_dict(rank0_only=True, offload_to_cpu=True)
        if rank == 0:
            os.makedirs(os.path.dirname(os.path.abspath(args.checkpoint)), exist_ok=True)
            torch.save({"model_state_dict": sd, "epoch": args.epochs}, args.checkpoint)
            print(f"[fsdp_unet] FULL_STATE_DICT ({len(sd)} tensors) -> {args.checkpoint}", flush=True)
    summary.update(example="fsdp_unet", world=world, params=n_params, sharding=args.sharding)
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
