#!/usr/bin/env python3
"""Domain (spatial) parallelism: one weather field split along latitude across ranks, halo-exchanging UNet.

Reference: documented only (docs/guide/10_domain_parallel.md:45-149: single-device halo demo with ``torch.cat``
padding, PhysicsNeMo ``ShardTensor`` recommended; scripts 07_domain_parallel_shardtensor/01..04 missing: X1).

Every rank holds rows [r*H/P, (r+1)*H/P) of each [B, C, H, W] field.  3x3 convolutions exchange one halo row
with their latitude neighbours (exact adjoint in backward), BatchNorm statistics are reduced over the domain
group, 2x2 pooling / transposed convolutions are shard-local (H/P divisible by 8), and the latitude weights of
the loss are the shard's slice of the global profile -- so the result equals training the unsharded UNet
(``--check`` verifies the first step's loss against a single-rank replay).  Weight gradients (partial sums of
each shard) are averaged over the group by the bucketed engine.  ``--dp`` > 1 adds data parallelism across
domain groups.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/07_domain_parallel/domain_parallel_unet.py \
        --lat 720 --lon 1440 --batch 1
"""
import copy
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_pytorch_hpc_amd.comm.mesh import Mesh  # noqa: E402
from distributed_pytorch_hpc_amd.models import SimpleUNet  # noqa: E402
from distributed_pytorch_hpc_amd.ops import latitude_weighted_mse  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.domain import convert_to_domain_parallel  # noqa: E402
from distributed_pytorch_hpc_amd.train.cli import common_parser, finish, start  # noqa: E402
from distributed_pytorch_hpc_amd.utils.metrics import sync  # noqa: E402


def main(argv=None):
    ap = common_parser(__doc__)
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2, help="fields per domain group")
    ap.add_argument("--channels", type=int, default=65)
    ap.add_argument("--lat", type=int, default=192)
    ap.add_argument("--lon", type=int, default=384)
    ap.add_argument("--base-dim", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--check", action="store_true", help="compare step-0 loss with an unsharded replay")
    # MIOpen find mode off by default here: the halo-padded slab shapes (and --check's unsharded replay) are new
    # convolution shapes for every layer, and a few-step fp32 run spends minutes timing solvers it never reuses.
    ap.set_defaults(conv_search=False)
    args = ap.parse_args(argv)
    rank, world, local, dev = start(args)
    assert world % args.dp == 0
    P = world // args.dp
    assert args.lat % (8 * P) == 0, "lat must split into shards divisible by 8 (3 pooling levels)"
    mesh = Mesh((args.dp, P), ("dp", "domain"))
    drank, dp_rank = mesh.local_rank("domain"), mesh.local_rank("dp")
    h = args.lat // P

    torch.manual_seed(args.seed)
    full_model = SimpleUNet(args.channels, args.channels, args.base_dim)
    ref = copy.deepcopy(full_model).to(dev) if args.check else None
    model = convert_to_domain_parallel(full_model, mesh.group("domain"), dim=2).to(dev)
    engine = DataParallelEngine(model, None, convert_linears=False)   # average over dp x domain ranks
    engine.configure_optimizer(OptimConfig("adamw", lr=args.lr, weight_decay=1e-5))
    times, losses = [], []
    for step in range(args.steps):
        g = torch.Generator(device=dev).manual_seed(1000 * step + dp_rank)
        x = torch.randn(args.batch, args.channels, args.lat, args.lon, device=dev, generator=g)
        y = torch.randn(args.batch, args.channels, args.lat, args.lon, device=dev, generator=g)
        xs, ys = x[:, :, drank * h:(drank + 1) * h].contiguous(), y[:, :, drank * h:(drank + 1) * h].contiguous()
        sync()
        t0 = time.perf_counter()
        loss = latitude_weighted_mse(model(xs), ys, n_lat_global=args.lat, lat_offset=drank * h)
        loss.backward()
        engine.step()
        engine.zero_grad()
        sync()
        times.append(time.perf_counter() - t0)
        lt = loss.detach().clone()
        dist.all_reduce(lt) if world > 1 else None
        losses.append(lt.item() / world)
        if step == 0 and ref is not None:
            with torch.no_grad():
                ref_loss = latitude_weighted_mse(ref(x), y).item()   # this dp group's full fields
            dl = loss.detach().clone()
            if P > 1:
                dist.all_reduce(dl, group=mesh.group("domain"))
            rel = abs(dl.item() / P - ref_loss) / max(abs(ref_loss), 1e-6)
            if rank == 0:
                print(f"step-0 loss sharded {dl.item() / P:.6f} vs unsharded {ref_loss:.6f} (rel {rel:.2e})",
                      flush=True)
            assert rel < 1e-4, rel
        if rank == 0:
            print(f"step {step}: loss {losses[-1]:.5f} | {1000 * times[-1]:.1f} ms", flush=True)
    engine.synchronize()
    steady = times[1:] if len(times) > 1 else times
    summary = {"example": "domain_parallel_unet", "domain": P, "dp": args.dp, "grid": [args.lat, args.lon],
               "shard_rows": h, "losses": losses, "ms_per_step": 1000 * sum(steady) / len(steady)}
    finish(args, summary, rank)


if __name__ == "__main__":
    main()
