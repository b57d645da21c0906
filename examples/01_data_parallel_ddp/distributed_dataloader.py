#!/usr/bin/env python3
"""DDP with a rank-sharded DataLoader: 2-layer MLP classifier on random features.

Reference: scripts/01_data_parallel_ddp/distributed_dataloader.py (SimpleDataset L143-156, SimpleModel L160-172,
SGD m=0.9, CrossEntropy, loss every 10 batches, average loss L267-278).  Rank discovery is the shared runtime
(runtime/env.py) instead of the script's private variant (reference defect X17).

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/01_data_parallel_ddp/distributed_dataloader.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch.nn.functional as F  # noqa: E402

from distributed_pytorch_hpc_amd.data import SimpleDataset, dp_dataloader  # noqa: E402
from distributed_pytorch_hpc_amd.models import SimpleModel  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP  # noqa: E402
from distributed_pytorch_hpc_amd.train import Trainer  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--dataset-size", type=int, default=1000)
    ap.add_argument("--input-dim", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--num-workers", type=int, default=0)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    ds = SimpleDataset(args.dataset_size, args.input_dim, seed=args.seed)
    loader, sampler = dp_dataloader(ds, args.batch_size, world, rank, shuffle=True, seed=args.seed,
                                    num_workers=args.num_workers)
    model = DDP(SimpleModel(args.input_dim).to(dev))
    opt = model.make_optimizer("sgd", lr=args.lr, momentum=0.9, weight_decay=0.0)
    trainer = Trainer(model, opt, loader, F.cross_entropy, dev, sampler=sampler, log_every=10,
                      metrics_file=args.metrics_file)
    summary = trainer.train(args.epochs)
    summary.update(example="distributed_dataloader", world=world,
                   samples_per_rank_per_epoch=len(sampler))
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
