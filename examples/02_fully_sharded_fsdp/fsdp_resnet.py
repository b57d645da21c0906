#!/usr/bin/env python3
"""FSDP ResNet-18 (CIFAR stem) with optional bf16 mixed precision; train loss/acc per epoch + collective test.

Reference: scripts/02_fully_sharded_fsdp/resnet_fsdp_training.py:158-241 (ResNet-18, conv1 3x3 s1, maxpool
Identity, 10 classes; ``size_based_auto_wrap_policy(min_num_params=1e5)``; ``ShardingStrategy.FULL_SHARD``;
``--use-amp`` -> ``MixedPrecision(param=bf16, reduce=bf16, buffer=bf16)``; SGD lr 0.01 m 0.9 wd 5e-4; CE;
Trainer.train_epoch / test L90-155).

With ``--data-dir`` pointing at the CIFAR-10 binary distribution (cifar-10-batches-bin) the real dataset is used:
held in HBM, batches gathered + augmented (RandomCrop(32, padding=4) + flip + Normalize, as the reference) on the
GPU by data/cifar.py.  Without it (no download here) batches are synthetic CIFAR-shaped tensors (3x32x32, 10
classes) generated on device.  Evaluation is collective (every rank scores its shard) so it
works under FSDP (reference defect X9).  ``--sharding`` selects FULL_SHARD / SHARD_GRAD_OP / NO_SHARD /
HYBRID_SHARD; ``--wrap`` size (default) or block (one unit per BasicBlock).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/02_fully_sharded_fsdp/fsdp_resnet.py --use-amp
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_pytorch_hpc_amd.data import CIFAR10, CIFARDeviceLoader, DeviceBatches  # noqa: E402
from distributed_pytorch_hpc_amd.models import resnet  # noqa: E402
from distributed_pytorch_hpc_amd.models.resnet import BasicBlock, Bottleneck  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import MixedPrecision  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.fsdp import (FSDP, ModuleWrapPolicy, ShardingStrategy,  # noqa: E402
                                                       size_based_auto_wrap_policy)
from distributed_pytorch_hpc_amd.train import Trainer  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--steps-per-epoch", type=int, default=20)
    ap.add_argument("--test-steps", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--image-size", type=int, default=32)
    ap.add_argument("--num-classes", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=5e-4)
    ap.add_argument("--use-amp", action="store_true", help="bf16 params / reduce / buffers")
    ap.add_argument("--sharding", default="FULL_SHARD", choices=[s.value for s in ShardingStrategy])
    ap.add_argument("--wrap", choices=["size", "block"], default="size")
    ap.add_argument("--min-num-params", type=int, default=int(1e5))
    ap.add_argument("--save-full-state", default=None, help="write the consolidated FULL_STATE_DICT here")
    ap.add_argument("--data-dir", default=None, help="CIFAR-10 binary distribution (cifar-10-batches-bin)")
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)

    model = resnet(args.arch, num_classes=args.num_classes, cifar_stem=True).to(dev)
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if args.use_amp else None
    policy = (size_based_auto_wrap_policy(args.min_num_params) if args.wrap == "size"
              else ModuleWrapPolicy({BasicBlock, Bottleneck}))
    fsdp = FSDP(model, sharding_strategy=args.sharding, mixed_precision=mp, auto_wrap_policy=policy)
    opt = fsdp.make_optimizer("sgd", lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    dtype = torch.bfloat16 if args.use_amp else torch.float32
    if args.data_dir:
        train = CIFARDeviceLoader(CIFAR10(args.data_dir, train=True), args.batch_size, dev, dp_rank=rank,
                                  dp_size=world, augment=True, seed=args.seed, dtype=dtype)
        test = CIFARDeviceLoader(CIFAR10(args.data_dir, train=False), args.batch_size, dev, dp_rank=rank,
                                 dp_size=world, augment=False, shuffle=False, drop_last=False, dtype=dtype)
    else:
        train = DeviceBatches("images", args.batch_size, dev, seed=args.seed, rank=rank, image_size=args.image_size,
                              num_classes=args.num_classes, dtype=dtype)
        test = DeviceBatches("images", args.batch_size, dev, seed=args.seed + 1, rank=rank,
                             image_size=args.image_size, num_classes=args.num_classes, dtype=dtype)

    def loss_fn(out, y):
        return F.cross_entropy(out.float(), y)

    trainer = Trainer(fsdp, opt, train, loss_fn, dev, max_steps_per_epoch=args.steps_per_epoch,
                      sampler=train if args.data_dir else None,
                      log_every=max(args.steps_per_epoch // 2, 1), metrics_file=args.metrics_file,
                      cuda_graph=args.cuda_graph)
    for epoch in range(args.epochs):
        st = trainer._run_epoch(epoch)
        trainer.history.append(st)
        ev = trainer.evaluate(test, max_steps=args.test_steps)
        if rank == 0:
            print(f"epoch {epoch}: train loss {st.loss:.4f} | test loss {ev['loss']:.4f} acc {ev['accuracy']:.4f} "
                  f"| {st.seconds:.2f}s | {st.samples_per_sec:.1f} img/s (global)", flush=True)
    summary = trainer.summary()
    if args.save_full_state:
        sd = fsdp.full_state_dict(rank0_only=True, offload_to_cpu=True)
        if rank == 0:
            torch.save(sd, args.save_full_state)
    summary.update(example="fsdp_resnet", world=world, sharding=args.sharding, amp=args.use_amp, test=ev)
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
