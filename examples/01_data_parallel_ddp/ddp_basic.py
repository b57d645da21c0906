#!/usr/bin/env python3
"""DDP basics: Linear(20 -> 1) regression with a resumable snapshot.

Reference: scripts/01_data_parallel_ddp/multinode_ddp_basic.py (Trainer L114-208, MyTrainDataset L89-105,
SGD lr 1e-3, MSE, DistributedSampler, ``snapshot.pt`` auto-resume, per-epoch + total/avg epoch time).

MI355X version: the bucketed all-reduce engine (parallel/data_parallel.py) instead of torch DDP, the fused SGD
kernel as the optimizer, and a single global-rank-0 snapshot writer (reference defect X15: one writer per node).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/01_data_parallel_ddp/ddp_basic.py 50 10
    python examples/01_data_parallel_ddp/ddp_basic.py 4 2 --device cpu        # single process
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch.nn.functional as F  # noqa: E402

from distributed_pytorch_hpc_amd.data import MyTrainDataset, dp_dataloader  # noqa: E402
from distributed_pytorch_hpc_amd.models import LinearModel  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP  # noqa: E402
from distributed_pytorch_hpc_amd.train import Trainer  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("total_epochs", type=int, nargs="?", default=5)
    ap.add_argument("save_every", type=int, nargs="?", default=2)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--dataset-size", type=int, default=2000)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--snapshot-path", default="snapshot.pt")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    ds = MyTrainDataset(args.dataset_size, seed=args.seed)
    loader, sampler = dp_dataloader(ds, args.batch_size, world, rank, shuffle=True, seed=args.seed, num_workers=0)
    model = DDP(LinearModel().to(dev))
    opt = model.make_optimizer("sgd", lr=args.lr, weight_decay=0.0)
    trainer = Trainer(model, opt, loader, F.mse_loss, dev, sampler=sampler, snapshot_path=args.snapshot_path,
                      save_every=args.save_every, log_every=0, metrics_file=args.metrics_file)
    summary = trainer.train(args.total_epochs)
    summary.update(example="ddp_basic", world=world, epoch_times=[round(h.seconds, 4) for h in trainer.history])
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
