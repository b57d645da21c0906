"""Pre-flight checks for multi-rank runs: exact collective self-test, cross-rank parameter agreement, and an
in-run alpha-beta probe of the collectives that sizes the gradient buckets.

Why: the first time a job meets real RCCL over xGMI (the round-end 8-GPU scaling run) a broken rank mapping, a
wrong HIP_VISIBLE_DEVICES, a mis-sized collective or a silently divergent replica must fail LOUDLY, before the timed
region, instead of hanging or publishing a number from diverged replicas.  The reference's equivalent is the
init-time NCCL smoke of ``tests/check_environment.py:76-109`` / ``utils/distributed.py:124-158`` and the timing loop
of ``tests/torch_comm_bench.py:32-116``; here the checks are exact (small integers, every element compared), bounded
by a timeout, and run on the job's own process group.

* ``collective_selftest`` -- all-reduce, reduce-scatter, all-gather (fp32 and bf16) and a P2P ring with known values.
* ``replicas_agree`` -- bitwise agreement of a flat parameter buffer across the replicas of a group (two
  order-sensitive float64 checksums, gathered and compared exactly).
* ``probe_alpha_beta`` -- a ~1-2 s sweep of reduce-scatter / all-gather at a few sizes, least-squares fitted
  (comm/cost_model.py) and turned into a bucket size with ``choose_bucket_bytes``.
"""
from __future__ import annotations

import datetime
from dataclasses import asdict

import torch
import torch.distributed as dist

from ..comm import cost_model


class PreflightError(RuntimeError):
    pass


def _wait(work, timeout_s: float, what: str):
    try:
        if work is None:
            return
        ok = work.wait(timeout=datetime.timedelta(seconds=timeout_s))
        if ok is False:
            raise PreflightError(f"{what}: timed out after {timeout_s:.0f} s")
    except PreflightError:
        raise
    except Exception as e:  # RCCL / gloo errors and timeouts surface here
        raise PreflightError(f"{what}: {type(e).__name__}: {e}") from e


def _dev_sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def collective_selftest(group=None, device=None, timeout_s: float = 120.0, numel: int = 1 << 16) -> dict:
    """Run every collective the engines use on ``group`` with values whose results are exact in bf16 and fp32, and
    compare every element.  Raises PreflightError naming the first failing collective; returns a small report."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    device = device or torch.device("cpu")
    if dist.get_backend(group) == "gloo":
        device = torch.device("cpu")   # gloo's transport is host memory (and its P2P takes CPU tensors only)
    report = {"world": world, "checked": []}
    n = max(world, numel // world * world)
    idx = torch.arange(n, device=device)
    for dtype in (torch.float32, torch.bfloat16):
        tag = str(dtype).replace("torch.", "")
        exact_sum = dtype == torch.float32
        if exact_sum:
            # all-reduce: rank r contributes (r + 1) * (1 + i % 4)  ->  sum = W(W+1)/2 * (1 + i % 4): exact in fp32 for
            # any realistic world (< 2^24), and it pins every rank's identity and the SUM reduction
            pattern = (idx % 4 + 1).to(dtype)
            x = pattern * (rank + 1)
            want = pattern * (world * (world + 1) // 2)
        else:
            # bf16: RCCL keeps partial sums in bf16 between hops, so only sums whose every partial sum has <= 8
            # significant bits are exact at any world size.  Element i gets a = 1 + i % 4 from rank i % W and 8 from
            # rank (i + 1) % W (zeros elsewhere): every partial sum is 0, a, 8 or a + 8, and SUM (not max / any single
            # contribution) is still what makes the total a + 8.
            a = (idx % 4 + 1).to(dtype)
            x = torch.where(idx % world == rank, a, torch.zeros_like(a)) + \
                torch.where((idx + 1) % world == rank, torch.full_like(a, 8), torch.zeros_like(a))
            want = a + 8
        _wait(dist.all_reduce(x, group=group, async_op=True), timeout_s, f"all_reduce[{tag}]")
        _dev_sync(device)
        if not torch.equal(x, want):
            bad = int((x != want).nonzero()[0])
            raise PreflightError(f"all_reduce[{tag}] mismatch on rank {rank}: element {bad} = {float(x[bad])}, "
                                 f"expected {float(want[bad])}")
        report["checked"].append(f"all_reduce[{tag}]")
        k = n // world
        chunk = torch.arange(world, device=device).repeat_interleave(k)
        if exact_sum:
            # reduce-scatter: input chunk c of rank r = (r + 1) * (c + 1)  ->  output of rank r = W(W+1)/2 * (r + 1)
            inp = (chunk + 1).to(dtype) * (rank + 1)
            want = torch.full((k,), float(world * (world + 1) // 2 * (rank + 1)), dtype=dtype, device=device)
        else:
            # bf16: chunk c gets 1 + (j + c) % 7 (element j) from rank c and 8 from rank (c + 1) % W: exact partial
            # sums, and the chunk -> rank order shows in the phase of the pattern
            j = torch.arange(n, device=device) % k
            inp = torch.where(chunk == rank, ((j + chunk) % 7 + 1).to(dtype), torch.zeros(n, dtype=dtype, device=device))
            inp = inp + torch.where((chunk + 1) % world == rank, torch.full((n,), 8.0, dtype=dtype, device=device),
                                    torch.zeros(n, dtype=dtype, device=device))
            want = ((torch.arange(k, device=device) + rank) % 7 + 9).to(dtype)
        out = torch.empty(k, dtype=dtype, device=device)
        _wait(dist.reduce_scatter_tensor(out, inp, group=group, async_op=True), timeout_s, f"reduce_scatter[{tag}]")
        _dev_sync(device)
        if not torch.equal(out, want):
            raise PreflightError(f"reduce_scatter[{tag}] mismatch on rank {rank}: got {float(out[0])} ... "
                                 f"expected {float(want[0])} (wrong rank order or reduction?)")
        report["checked"].append(f"reduce_scatter[{tag}]")
        # all-gather: rank r contributes r + 1 in every element  ->  chunk c == c + 1
        src = torch.full((k,), float(rank + 1), dtype=dtype, device=device)
        full = torch.empty(k * world, dtype=dtype, device=device)
        _wait(dist.all_gather_into_tensor(full, src, group=group, async_op=True), timeout_s, f"all_gather[{tag}]")
        _dev_sync(device)
        want = (torch.arange(world, device=device).repeat_interleave(k) + 1).to(dtype)
        if not torch.equal(full, want):
            bad = int((full != want).nonzero()[0])
            raise PreflightError(f"all_gather[{tag}] mismatch on rank {rank}: chunk {bad // k} holds "
                                 f"{float(full[bad])}, expected {bad // k + 1}")
        report["checked"].append(f"all_gather[{tag}]")
    # P2P ring: send rank id to the next rank, receive from the previous one (both directions of every xGMI link
    # the ring uses are exercised at world >= 3; world 2 is a ping-pong)
    if world > 1:
        g_rank = lambda r: dist.get_global_rank(group, r) if group is not None else r  # noqa: E731
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        s = torch.full((1024,), float(rank), device=device)
        r = torch.empty(1024, device=device)
        ops = [dist.P2POp(dist.isend, s, g_rank(nxt), group), dist.P2POp(dist.irecv, r, g_rank(prv), group)]
        for w in dist.batch_isend_irecv(ops):
            _wait(w, timeout_s, "p2p ring")
        _dev_sync(device)
        if not torch.all(r == float(prv)):
            raise PreflightError(f"p2p ring mismatch on rank {rank}: received {float(r[0])}, expected {prv}")
        report["checked"].append("p2p_ring")
    return report


def checksum(flat: torch.Tensor, chunk: int = 1 << 26) -> torch.Tensor:
    """Two order-sensitive float64 checksums of a flat tensor: plain sum and a position-weighted sum (a swapped pair
    of elements changes the second).  Chunked: a 7B-parameter buffer as one float64 copy would need 54 GB."""
    x = flat.detach().reshape(-1)
    acc = torch.zeros(2, dtype=torch.float64, device=x.device)
    for o in range(0, x.numel(), chunk):
        c = x[o:o + chunk].double()
        w = (torch.arange(o, o + c.numel(), device=x.device, dtype=torch.int64) % 1021 + 1).double()
        acc[0] += c.sum()
        acc[1] += (c * w).sum()
    return acc


def replicas_agree(flat: torch.Tensor, group=None, timeout_s: float = 120.0) -> dict:
    """Gather ``checksum(flat)`` from every rank of ``group`` (ranks holding replicas of the same parameters) and
    require bitwise equality.  Raises PreflightError with the per-rank values on divergence."""
    world = dist.get_world_size(group)
    c = checksum(flat)
    allc = torch.empty(world, 2, dtype=torch.float64, device=c.device)
    _wait(dist.all_gather_into_tensor(allc, c.reshape(1, 2), group=group, async_op=True), timeout_s,
          "parameter checksum all_gather")
    vals = allc.cpu().tolist()
    ok = all(v == vals[0] for v in vals)
    if not ok:
        raise PreflightError(f"replicas diverged: per-rank parameter checksums {vals}")
    return {"ok": True, "checksum": vals[0]}


def probe_alpha_beta(group=None, device=None, sizes_mib=(4, 16, 64, 256), dtype=torch.bfloat16, iters: int = 3,
                     budget_s: float = 2.0) -> dict:
    """Time reduce-scatter and all-gather on ``group`` at ``sizes_mib`` (message size per rank in the rccl-tests
    convention), fit alpha-beta per op and return {op: AlphaBeta}.  Sizes whose first call alone exceeds the budget
    stop the sweep (slow backends, e.g. gloo on CPU: the fit then uses the smaller sizes)."""
    world = dist.get_world_size(group)
    fits = {}
    # The stop decision must be identical on every rank (a rank that skips a size while the others enter its
    # collective deadlocks the job), so it is taken on the measured times -- measure() returns the slowest rank's
    # time, the same value everywhere -- never on a rank-local wall clock.
    spent = 0.0
    for op in ("reduce_scatter", "all_gather"):
        samples = []
        for mib in sizes_mib:
            if samples and spent > budget_s:
                break
            got = cost_model.measure(op, [int(mib * 2 ** 20)], group=group, device=device, dtype=dtype,
                                     iters=iters, warmup=1)
            spent += sum(t for _, t in got) * (iters + 1)
            samples += got
        if len(samples) < 2:   # need two points for a slope; fall back to the smallest extra size
            samples += cost_model.measure(op, [int(2 * sizes_mib[0] * 2 ** 20)], group=group, device=device,
                                          dtype=dtype, iters=iters, warmup=1)
        fits[op] = cost_model.fit_alpha_beta(op, world, samples)
        fits[op].source = f"in-run probe ({len(samples)} sizes)"
    return fits


def calibrated_bucket_mb(fits: dict, grad_bytes: float, sharded: bool, lo_mib: float = 32.0,
                         hi_mib: float = 512.0) -> float:
    """Bucket size (MiB) from the probe's fit (reduce-scatter for the sharded engine, all-reduce ~ 2x reduce-scatter
    bytes otherwise), clamped to [lo, hi] so a noisy fit cannot produce a pathological partition."""
    m = fits["reduce_scatter"]
    if not sharded:
        m = cost_model.AlphaBeta("all_reduce", m.world, m.alpha_s, m.beta_bus_Bps, m.source)
    mib = cost_model.choose_bucket_bytes(m, grad_bytes) / 2 ** 20
    return float(min(max(mib, lo_mib), hi_mib))


def fits_json(fits: dict) -> dict:
    return {k: {kk: (round(vv, 9) if isinstance(vv, float) else vv) for kk, vv in asdict(v).items()}
            for k, v in fits.items()}


def rccl_version() -> str | None:
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None
