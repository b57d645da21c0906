"""Worker of tests/test_multigpu.py: one rank per GPU over RCCL (runtime/launch.py --nproc W), distinct devices.

    python -m distributed_pytorch_hpc_amd.runtime.launch --nproc W --cpu-bind none tests/scripts/multigpu_worker.py CASE

CASE is one of
  collectives  all-reduce / all-gather / reduce-scatter / all-to-all / send-recv ring / broadcast on exact integer
               data (fp32, bf16, int64) -- RCCL over xGMI, every result compared bit-for-bit with its known value;
  xgmi         the direct-peer IPC all-reduce (csrc/custom_allreduce.hip) across DISTINCT devices: bitwise equal to
               RCCL on integer-valued data and to a host fp32 rank-order sum on random data, one- and two-shot,
               in place and out of place, then the probe's crossover and the stream-ordered step guard;
  tp           Llama TP = W (+ SP, loss parallel, async TP) vs a one-rank run of the same model and batch (bf16, HIP
               kernels), 3 AdamW steps: losses and re-assembled weights;
  pp           PP = W (1F1B) vs the one-rank step: loss and every gradient.
Every rank prints nothing but failures; rank 0 ends with ``MGPU_RESULT case=... world=W failures=N`` and the job exits
non-zero if any rank failed.  (Reference: tests/torch_comm_bench.py:40-89 times the same collectives without checking
them; tests/pbs_run_tests.sh:128-158 runs them under mpiexec.)
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402

PRESET = dict(dim=256, n_layers=2, n_heads=8, vocab_size=512, max_seq_len=256, multiple_of=64)


def _eq(fails, what, got, want):
    if not torch.equal(got.cpu(), want.cpu()):
        bad = (got.float().cpu() - want.float().cpu()).abs().max().item()
        fails.append(f"{what}: max |err| {bad}")


def case_collectives(rank, world, dev):
    fails = []
    for dtype in (torch.float32, torch.bfloat16, torch.int64):
        n = 840 * 64          # divisible by every world size 1..8
        # integer data whose every partial sum stays exact: bf16 holds integers exactly up to 256 (world 8: 8 x 22 + 28)
        base = torch.arange(n, device=dev) % (23 if dtype == torch.bfloat16 else 97)
        x = (base + rank).to(dtype)
        dist.all_reduce(x)
        _eq(fails, f"all_reduce[{dtype}]", x, (world * base + world * (world - 1) // 2).to(dtype))
        mx = torch.full((n,), float(rank), device=dev).to(dtype)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        _eq(fails, f"all_reduce max[{dtype}]", mx, torch.full((n,), float(world - 1), device=dev).to(dtype))
        shard = (base[: n // world] + 1000 * rank).to(dtype) if dtype != torch.bfloat16 else \
            (base[: n // world] + rank).to(dtype)
        full = torch.empty(n // world * world, dtype=dtype, device=dev)
        dist.all_gather_into_tensor(full, shard)
        want = torch.cat([(base[: n // world] + (1000 * r if dtype != torch.bfloat16 else r)) for r in range(world)])
        _eq(fails, f"all_gather[{dtype}]", full, want.to(dtype))
        inp = (torch.arange(n, device=dev) % 13 + rank).to(dtype)
        out = torch.empty(n // world, dtype=dtype, device=dev)
        dist.reduce_scatter_tensor(out, inp)
        want = (world * (torch.arange(n, device=dev) % 13) + world * (world - 1) // 2)[rank * (n // world):
                                                                                      (rank + 1) * (n // world)]
        _eq(fails, f"reduce_scatter[{dtype}]", out, want.to(dtype))
        a2a_in = (torch.arange(world * 64, device=dev) // 64 * 10 + rank).to(dtype)   # chunk j -> rank j
        a2a_out = torch.empty_like(a2a_in)
        dist.all_to_all_single(a2a_out, a2a_in)
        want = (rank * 10 + torch.arange(world * 64, device=dev) // 64).to(dtype)      # chunk j came from rank j
        _eq(fails, f"all_to_all[{dtype}]", a2a_out, want)
        b = torch.full((1024,), float(rank + 5), device=dev).to(dtype)
        dist.broadcast(b, src=world - 1)
        _eq(fails, f"broadcast[{dtype}]", b, torch.full((1024,), float(world + 4), device=dev).to(dtype))
    # send / recv ring, both directions (even ranks send first)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    for direction in (1, -1):
        to, frm = (nxt, prv) if direction == 1 else (prv, nxt)
        s = torch.full((4096,), float(rank), device=dev)
        r = torch.empty_like(s)
        ops = [dist.P2POp(dist.isend, s, to), dist.P2POp(dist.irecv, r, frm)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        _eq(fails, f"p2p ring dir {direction}", r, torch.full((4096,), float(frm), device=dev))
    if world > 1:
        s = torch.full((777,), float(rank), device=dev)
        if rank % 2 == 0 and rank + 1 < world:
            dist.send(s, rank + 1)
        elif rank % 2 == 1:
            r = torch.empty_like(s)
            dist.recv(r, rank - 1)
            _eq(fails, "send/recv pair", r, torch.full((777,), float(rank - 1), device=dev))
    torch.cuda.synchronize()
    return fails


def case_xgmi(rank, world, dev):
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as C

    fails = []
    car = C.XgmiAllReduce(None, max_bytes=8 << 20)
    case = 0
    for dtype in (torch.float32, torch.bfloat16):
        for algo in ("oneshot", "twoshot", "auto"):
            for n in (8, 4104, 65536 + 24, 1 << 20):
                if n * torch.empty((), dtype=dtype).element_size() > car.max_bytes:
                    continue
                case += 1
                # integer-valued: every summation order is exact, so RCCL and the direct-peer path agree bitwise
                xi = (torch.arange(n, device=dev) % 25 + rank).to(dtype)   # world-8 sums <= 220: exact in bf16
                ref = xi.clone()
                dist.all_reduce(ref)
                got = car.all_reduce(xi.clone(), algo=algo) if case % 2 else \
                    car.all_reduce(xi, algo=algo, out=torch.empty_like(xi))
                _eq(fails, f"xgmi vs rccl {dtype} {algo} n={n}", got, ref)
                # random: the kernel's contract is the fp32 rank-order sum, identical on every rank
                g = torch.Generator().manual_seed(1000 * case + rank)
                xr = torch.randn(n, generator=g).to(dtype)
                xs = [None] * world
                dist.all_gather_object(xs, xr)
                want = torch.zeros(n)
                for t in xs:
                    want = want + t.float()
                got = car.all_reduce(xr.to(dev), algo=algo)
                _eq(fails, f"xgmi rank-order sum {dtype} {algo} n={n}", got, want.to(dtype))
    if car.errors():
        fails.append(f"{car.errors()} barrier timeouts")
    car.close()
    res = C.probe_crossover(None)
    if not res["verified"]:
        fails.append(f"crossover probe failed verification: {res}")
    if rank == 0:
        print(f"xgmi crossover {res['crossover_bytes']} B; samples (bytes, rccl s, xgmi s): {res['samples']}",
              flush=True)
    # the stream-ordered step guard on a healthy group: the scale stays finite, no error is reported
    gs = torch.ones(1, device=dev)
    C.guard_update(gs)
    C.check_health()
    torch.cuda.synchronize()
    if not torch.isfinite(gs).all():
        fails.append("guard poisoned the scale of a healthy group")
    C.drop(None)
    return fails


def _llama(dev, seed=7):
    from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama

    return build_llama(ModelArgs(**PRESET), device=dev, dtype=torch.bfloat16, seed=seed)


def _batches(steps=3, b=4, s=128):
    g = torch.Generator().manual_seed(3)
    return [torch.randint(0, PRESET["vocab_size"], (b, s + 1), generator=g) for _ in range(steps)]


def _train(m, eng, batches, dev):
    losses = []
    for t in batches:
        t = t.to(dev)
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        eng.step()
        eng.zero_grad()
        losses.append(float(loss.detach().float()))
    eng.synchronize()
    torch.cuda.synchronize()
    return losses


def case_tp(rank, world, dev):
    from distributed_pytorch_hpc_amd.comm.mesh import DeviceMesh2D
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama

    fails = []
    solo = DeviceMesh2D(world, 1)   # dp = world, tp = 1: tp_group is this rank alone (the one-rank reference)
    mesh = DeviceMesh2D(1, world)
    batches = _batches()
    ref = _llama(dev)
    eng = DataParallelEngine(ref, process_group=solo.tp_group, shard=False)
    eng.configure_optimizer(OptimConfig(lr=1e-3, weight_decay=0.1))
    ref_losses = _train(ref, eng, batches, dev)
    ref_sd = {k: v.detach().float().cpu() for k, v in ref.state_dict().items()}
    for async_tp in (0, 2):
        m = _llama(dev)
        parallelize_llama(m, mesh.tp_group, sequence_parallel=True, loss_parallel=True, async_tp=async_tp)
        eng = DataParallelEngine(m, process_group=mesh.dp_group, shard=False)
        eng.configure_optimizer(OptimConfig(lr=1e-3, weight_decay=0.1))
        losses = _train(m, eng, batches, dev)
        for a, b in zip(ref_losses, losses):
            if abs(a - b) > 2e-2 * max(1.0, abs(a)):
                fails.append(f"async_tp={async_tp}: losses {losses} vs one rank {ref_losses}")
                break
        sd = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
        parts = [None] * world
        dist.all_gather_object(parts, {k: sd[k] for k in ("layers.0.feed_forward.w2.weight",
                                                          "layers.1.attention.wo.weight", "tok_embeddings.weight")})
        checks = {"layers.0.feed_forward.w2.weight": 1, "layers.1.attention.wo.weight": 1,
                  "tok_embeddings.weight": 0}
        for k, d in checks.items():
            full = torch.cat([p[k] for p in parts], d)
            err = (full - ref_sd[k]).norm() / ref_sd[k].norm()
            if not err < 2e-2:
                fails.append(f"async_tp={async_tp}: {k} rel err {err:.3e} vs the one-rank run")
        norm_err = (sd["layers.0.ffn_norm.weight"] - ref_sd["layers.0.ffn_norm.weight"]).abs().max()
        if not norm_err < 2e-2:
            fails.append(f"async_tp={async_tp}: SP norm weight max err {norm_err:.3e}")
    return fails


def case_pp(rank, world, dev):
    from distributed_pytorch_hpc_amd.parallel.pipeline import PipelineSchedule, lm_loss, split_llama

    fails = []
    micro = 4
    t = _batches(1, b=8, s=64)[0].to(dev)
    x, y = t[:, :-1], t[:, 1:]
    ref = _llama(dev, seed=11)
    names = {id(p): n for n, p in ref.named_parameters()}
    total = 0.0
    for xm, ym in zip(x.chunk(micro), y.chunk(micro)):
        loss = lm_loss(ref(xm), ym) / micro
        loss.backward()
        total += float(loss.detach().float())
    ref_g = {names[id(p)]: (p.main_grad if getattr(p, "main_grad", None) is not None else p.grad).float().clone()
             for p in ref.parameters()}
    model = _llama(dev, seed=11)
    names = {id(p): n for n, p in model.named_parameters()}
    sm = split_llama(model, world, rank)
    sched = PipelineSchedule(sm, rank, world, micro, loss_fn=lm_loss, group=None, schedule="1f1b")
    losses = sched.step(inputs=x if rank == 0 else None, target=y if rank == world - 1 else None)
    torch.cuda.synchronize()
    if rank == world - 1:
        got = sum(float(v) for v in losses) / micro
        if abs(got - total) > 2e-2 * max(1.0, abs(total)):
            fails.append(f"pp loss {got} vs one rank {total}")
    for p in sm.parameters():
        g = (p.main_grad if getattr(p, "main_grad", None) is not None else p.grad).float()
        r = ref_g[names[id(p)]]
        err = (g - r).norm() / r.norm().clamp_min(1e-12)
        if not err < 3e-2:
            fails.append(f"pp grad {names[id(p)]}: rel err {err:.3e}")
    return fails


CASES = {"collectives": case_collectives, "xgmi": case_xgmi, "tp": case_tp, "pp": case_pp}


def main():
    case = sys.argv[1]
    rank, world, local = rt.init_distributed(backend="nccl", verbose=False)
    dev = torch.device("cuda", local)
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    try:
        fails = CASES[case](rank, world, dev)
    except Exception as e:  # reported, then the gang exits non-zero
        import traceback

        fails = [f"exception: {e!r}\n{traceback.format_exc()}"]
    allf = [None] * world
    dist.all_gather_object(allf, fails)
    if rank == 0:
        flat = [f"rank{r}: {m}" for r, fl in enumerate(allf) for m in fl]
        print(f"MGPU_RESULT case={case} world={world} failures={len(flat)}", flush=True)
        for m in flat[:30]:
            print(m, flush=True)
    rt.cleanup_distributed()
    sys.exit(1 if any(allf) else 0)


if __name__ == "__main__":
    main()
