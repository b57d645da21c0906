"""Worker for tests/test_custom_allreduce.py: N processes share ONE GPU (the test box has one), exchange IPC handles
over gloo and run the direct-peer-read all-reduce; every rank checks bit-exact results against a host-side fp32
rank-order sum.  Launched by torch.distributed.run with --nproc-per-node N."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_pytorch_hpc_amd.comm.custom_allreduce import XgmiAllReduce  # noqa: E402


def inputs(world, case, numel, dtype):
    xs = []
    for r in range(world):
        g = torch.Generator().manual_seed(1000 * case + r)
        xs.append(torch.randn(numel, generator=g).to(dtype))
    return xs


def expected(xs, scale):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:
        acc = acc + x.float()
    return (acc * scale).to(xs[0].dtype)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    car = XgmiAllReduce(None, max_bytes=8 << 20, timeout_s=20.0, max_blocks=int(os.environ.get("CAR_BLOCKS", "16")))
    sizes = [8, 256, 4104, 65536 + 24, 1 << 20, (3 << 20) // 2]
    case = 0
    fails = []
    for dtype in (torch.float32, torch.bfloat16):
        for algo in ("oneshot", "twoshot", "auto"):
            for n in sizes:
                if n * (4 if dtype == torch.float32 else 2) > car.max_bytes or (n * (4 if dtype == torch.float32 else 2)) % 16:
                    continue
                for op in ("sum", "avg"):
                    case += 1
                    xs = inputs(world, case, n, dtype)
                    want = expected(xs, 1.0 / world if op == "avg" else 1.0)
                    t = xs[rank].cuda()
                    inplace = case % 2 == 0
                    out = car.all_reduce(t, op=op, algo=algo) if inplace else \
                        car.all_reduce(t, op=op, algo=algo, out=torch.empty_like(t))
                    got = out.cpu()
                    if not torch.equal(got, want):
                        bad = (got.float() - want.float()).abs().max().item()
                        fails.append(f"{dtype} {algo} n={n} op={op} inplace={inplace}: max err {bad}")
    # HIP graph: the per-block epochs advance on the device, so replays stay in step across ranks
    x = torch.full((4096,), float(rank + 1), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = torch.empty_like(x)
        car.all_reduce(x, out=y)            # warm-up outside capture
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            car.all_reduce(x, out=y)
    torch.cuda.current_stream().wait_stream(s)
    for i in range(3):
        x.fill_(float(i + rank))
        graph.replay()
        torch.cuda.synchronize()
        want = float(sum(i + r for r in range(world)))
        if not torch.all(y == want):
            fails.append(f"graph replay {i}: got {y[:4].tolist()} want {want}")
    err = car.errors()
    if err:
        fails.append(f"{err} barrier timeouts")
    car.close()
    flags = [None] * world
    dist.all_gather_object(flags, fails)
    if rank == 0:
        allf = [f"rank{r}: {m}" for r, fl in enumerate(flags) for m in fl]
        print(f"CAR_RESULT world={world} cases={case} failures={len(allf)}")
        for m in allf[:20]:
            print(m)
    dist.destroy_process_group()
    sys.exit(1 if any(flags) else 0)


if __name__ == "__main__":
    main()
