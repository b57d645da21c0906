#!/usr/bin/env python3
"""DDP UNet on ERA5-shaped synthetic fields with latitude-weighted MSE; reports global samples/s.

Reference: scripts/01_data_parallel_ddp/multinode_ddp_unet.py:236-404 (SimpleUNet 65->65 channels on 181x360,
batch 4, AdamW lr 1e-4 wd 1e-5, latitude-weighted MSE, per-batch / per-epoch / total samples/s, per-GPU rate).

MI355X version: batches are generated ON DEVICE (the reference builds ``randn(65,181,360)`` twice per sample on
CPU workers, defect X16: loader-bound), gradients go through the bucketed RCCL all-reduce engine, the optimizer
is the fused AdamW kernel, ``--amp`` runs the convolutions in bf16 autocast, ``--channels-last`` uses NHWC.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/01_data_parallel_ddp/ddp_unet.py --epochs 3
    python examples/01_data_parallel_ddp/ddp_unet.py --device cpu --lat 32 --lon 64 --steps-per-epoch 2
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from distributed_pytorch_hpc_amd.data import DeviceBatches  # noqa: E402
from distributed_pytorch_hpc_amd.models import SimpleUNet  # noqa: E402
from distributed_pytorch_hpc_amd.models.unet import to_channels_last  # noqa: E402
from distributed_pytorch_hpc_amd.ops import latitude_weighted_mse  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP  # noqa: E402
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
    ap.add_argument("--amp", action="store_true", help="bf16 autocast")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--snapshot-path", default=None)
    ap.add_argument("--save-every", type=int, default=0)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    model = SimpleUNet(args.channels, args.channels, args.base_dim).to(dev)
    if args.channels_last:
        model = to_channels_last(model)
    ddp = DDP(model)
    opt = ddp.make_optimizer("adamw", lr=args.lr, weight_decay=args.weight_decay)
    data = DeviceBatches("era5", args.batch_size, dev, seed=args.seed, rank=rank, channels=args.channels,
                         lat=args.lat, lon=args.lon)
    if rank == 0:
        n = sum(p.numel() for p in model.parameters())
        print(f"[ddp_unet] {n:,} params, world {world}, per-rank batch {args.batch_size}, grid {args.lat}x{args.lon}")
    trainer = Trainer(ddp, opt, data, latitude_weighted_mse, dev, max_steps_per_epoch=args.steps_per_epoch,
                      log_every=max(args.steps_per_epoch // 4, 1),
                      autocast_dtype=torch.bfloat16 if args.amp else None, snapshot_path=args.snapshot_path,
                      save_every=args.save_every, metrics_file=args.metrics_file,
                      cuda_graph=args.cuda_graph)
    summary = trainer.train(args.epochs)
    summary.update(example="ddp_unet", world=world, params=sum(p.numel() for p in model.parameters()))
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
