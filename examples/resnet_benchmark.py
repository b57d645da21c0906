#!/usr/bin/env python3
"""ResNet-18/50/101/152 data-parallel benchmark (DDP or FSDP), synthetic ImageNet-shaped batches.

Reference: scripts/main.py:117-399 (torchvision ``--arch resnet{18,50,101,152}``, ``--use_syn`` fixed
rand(B, 3, 224, 224) batch reused for ``--steps_syn 20`` steps per epoch, or CIFAR-10; ``--use_fsdp``; SGD lr 0.1
m 0.9 wd 1e-5; ``--resume``; average epoch time excluding epoch 0, appended with the torch config and NCCL
version to ``--logfile resnet_benchmark.log``).  It is the reference's only ResNet-50 benchmark path and the
source of two BASELINE.json configs: ResNet-50 DDP on CPU/gloo (world 2) and ResNet-50 FSDP bf16 on 8 GPUs.

MI355X version: ResNets defined natively (torchvision is not installed), channels-last bf16 convolutions
through MIOpen under ``--amp``, gradient buckets on the RCCL engine (``--ddp``) or sharded FSDP units
(``--use-fsdp``, bf16 MixedPrecision with ``--amp``), evaluation collective on every rank (reference X9: rank-0
eval hangs under FSDP).  ``--data-dir`` trains on CIFAR-10 from its binary distribution (no download here): the
dataset sits in HBM and batches are gathered + augmented on the GPU (data/cifar.py); otherwise ``--use-syn``.

    python examples/resnet_benchmark.py --device cpu --arch resnet50 --batch-size 8 --epochs 2 --steps-syn 2
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/resnet_benchmark.py --use-fsdp --amp --channels-last
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_pytorch_hpc_amd.data import CIFAR10, CIFARDeviceLoader, DeviceBatches  # noqa: E402
from distributed_pytorch_hpc_amd.models import resnet  # noqa: E402
from distributed_pytorch_hpc_amd.models.resnet import BasicBlock, Bottleneck  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DDP, MixedPrecision  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP, ModuleWrapPolicy  # noqa: E402
from distributed_pytorch_hpc_amd.train import Trainer  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402


def env_report(backend: str) -> str:
    lines = [f"torch {torch.__version__}", f"hip {getattr(torch.version, 'hip', None)}", f"backend {backend}"]
    if torch.cuda.is_available():
        try:
            v = torch.cuda.nccl.version()
            lines.append("rccl " + ".".join(str(x) for x in v) if isinstance(v, tuple) else f"rccl {v}")
        except Exception:  # noqa: BLE001
            pass
        lines.append(f"gpu {torch.cuda.get_device_name()}")
    return " | ".join(lines)


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--arch", default="resnet50", choices=["resnet18", "resnet50", "resnet101", "resnet152"])
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=256, help="per rank")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--use-syn", action="store_true", default=True)
    ap.add_argument("--steps-syn", type=int, default=20, help="synthetic steps per epoch")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=1e-5)
    ap.add_argument("--use-fsdp", action="store_true")
    ap.add_argument("--amp", action="store_true", help="bf16 (autocast for DDP, MixedPrecision for FSDP)")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--resume", default=None, help="snapshot path (DDP): resume from / save to")
    ap.add_argument("--logfile", default=None, help="append a result line (reference: resnet_benchmark.log)")
    ap.add_argument("--eval-steps", type=int, default=0)
    ap.add_argument("--data-dir", default=None, help="CIFAR-10 binary distribution (cifar-10-batches-bin): real data, "
                                                     "full epochs, 10 classes")
    args = ap.parse_args(argv)
    if args.data_dir:
        args.use_syn, args.num_classes = False, 10
    rank, world, local, dev = start(args)   # MIOpen find mode on GPU unless --no-conv-search (train/cli.py)
    backend = dist.get_backend() if dist.is_initialized() else ("nccl" if dev.type == "cuda" else "gloo")

    torch.manual_seed(args.seed)
    model = resnet(args.arch, num_classes=args.num_classes).to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    n_params = sum(p.numel() for p in model.parameters())
    autocast = None
    in_dtype = torch.float32
    if args.use_fsdp:
        mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if args.amp else None
        wrapped = FSDP(model, mixed_precision=mp, auto_wrap_policy=ModuleWrapPolicy({BasicBlock, Bottleneck}))
        in_dtype = torch.bfloat16 if args.amp else torch.float32
    else:
        wrapped = DDP(model)
        autocast = torch.bfloat16 if args.amp else None
    opt = wrapped.make_optimizer("sgd", lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    data = DeviceBatches("images", args.batch_size, dev, seed=args.seed, rank=rank, image_size=args.image_size,
                         num_classes=args.num_classes, dtype=in_dtype, fixed=True)
    cifar = test = None
    if args.data_dir:
        cifar = CIFARDeviceLoader(CIFAR10(args.data_dir, train=True), args.batch_size, dev, dp_rank=rank,
                                  dp_size=world, seed=args.seed, dtype=in_dtype, channels_last=args.channels_last)
        test = CIFARDeviceLoader(CIFAR10(args.data_dir, train=False), args.batch_size, dev, dp_rank=rank,
                                 dp_size=world, augment=False, shuffle=False, drop_last=False, dtype=in_dtype,
                                 channels_last=args.channels_last)

    class _CL:
        """channels-last view of the synthetic stream"""

        def __iter__(self):
            return self

        def __next__(self):
            x, y = next(data)
            return (x.contiguous(memory_format=torch.channels_last) if args.channels_last else x), y

    def loss_fn(out, y):
        return F.cross_entropy(out.float(), y)

    trainer = Trainer(wrapped, opt, cifar if cifar is not None else _CL(), loss_fn, dev,
                      max_steps_per_epoch=None if cifar is not None else args.steps_syn, sampler=cifar,
                      log_every=max(args.steps_syn // 2, 1), autocast_dtype=autocast,
                      snapshot_path=args.resume if not args.use_fsdp else None,
                      save_every=1 if args.resume and not args.use_fsdp else 0, metrics_file=args.metrics_file,
                      cuda_graph=args.cuda_graph)
    if rank == 0:
        print(f"[resnet_benchmark] {args.arch} {n_params:,} params | world {world} | "
              f"{'FSDP' if args.use_fsdp else 'DDP'} | per-rank batch {args.batch_size} | {env_report(backend)}",
              flush=True)
    summary = trainer.train(args.epochs)
    if args.eval_steps:
        summary["eval"] = trainer.evaluate(test if test is not None else _CL(), max_steps=args.eval_steps)
    summary.update(example="resnet_benchmark", arch=args.arch, params=n_params, world=world,
                   mode="fsdp" if args.use_fsdp else "ddp", amp=args.amp,
                   images_per_sec=summary["samples_per_sec_excl_first"] or summary["samples_per_sec"])
    if rank == 0 and args.logfile:
        with open(args.logfile, "a") as fh:
            fh.write(f"{time.strftime('%Y-%m-%d %H:%M:%S')} {args.arch} world={world} "
                     f"{'fsdp' if args.use_fsdp else 'ddp'} amp={args.amp} bs={args.batch_size} "
                     f"avg_epoch_s(excl 0)={summary['avg_epoch_seconds_excl_first']:.4f} "
                     f"img/s(excl 0)={summary['images_per_sec']:.1f} | {env_report(backend)}\n")
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
