"""alpha-beta cost model of the collectives, fitted from measurements, and the bucket sizes it implies.

SURVEY.md 7.1 item 4 / 7.7: "choose B so that alpha <= ~10 % of t(B) while keeping >= 3-4 buckets in flight during
backward", with t(B) = alpha + f(n) * B / beta_bus, where f(n) is the collective's bus factor (rccl-tests convention:
all-reduce 2(n-1)/n, all-gather / reduce-scatter / all-to-all (n-1)/n) and beta_bus the bus bandwidth the algorithm
sustains.  On an 8 x MI355X node a single RCCL ring is bounded by one xGMI link (~153 GB/s); algorithms that drive
several links at once (RCCL multi-channel, the direct-peer all-reduce of comm/custom_allreduce.py) exceed it -- so
the numbers must be MEASURED on the node (``benchmarks/comm_bench.py --fit fit.json``) rather than copied from the
reference's NVLink/Slingshot defaults (25 MiB DDP buckets).

The reference has no cost model; it never sets ``bucket_cap_mb`` (SURVEY.md S-DDP).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass

import torch
import torch.distributed as dist

BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
}


@dataclass
class AlphaBeta:
    op: str
    world: int
    alpha_s: float          # per-call latency
    beta_bus_Bps: float     # sustained bus bandwidth (bytes/s)
    source: str = "fit"

    def time(self, nbytes: float) -> float:
        n = max(self.world, 2)
        return self.alpha_s + BUS_FACTOR[self.op](n) * nbytes / self.beta_bus_Bps


def fit_alpha_beta(op: str, world: int, samples: list[tuple[float, float]]) -> AlphaBeta:
    """Least-squares fit of t = alpha + f * bytes / beta over ``samples`` = [(bytes, seconds), ...].
    Non-physical fits (negative alpha or slope) are clamped: alpha >= 0, beta from the largest message."""
    assert samples, "no samples"
    f = BUS_FACTOR[op](max(world, 2))
    xs = [f * b for b, _ in samples]
    ts = [t for _, t in samples]
    n = len(xs)
    mx, mt = sum(xs) / n, sum(ts) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    slope = sum((x - mx) * (t - mt) for x, t in zip(xs, ts)) / sxx if sxx > 0 else 0.0
    alpha = mt - slope * mx
    if slope <= 0 or alpha < 0:
        b_big, t_big = max(samples)
        alpha = max(0.0, min(ts))
        slope = max((t_big - alpha) / (f * b_big), 1e-15)
    return AlphaBeta(op, world, alpha, 1.0 / slope)


def choose_bucket_bytes(model: AlphaBeta, total_bytes: float, alpha_frac: float = 0.1, min_buckets: int = 4,
                        granule: int = 1 << 20) -> int:
    """Smallest bucket with alpha <= alpha_frac * t(B), but no larger than total / min_buckets (so several
    buckets are in flight while backward still produces gradients).  Rounded up to ``granule`` bytes."""
    f = BUS_FACTOR[model.op](max(model.world, 2))
    b_latency = model.alpha_s * (1.0 - alpha_frac) / alpha_frac * model.beta_bus_Bps / f
    b_overlap = total_bytes / max(min_buckets, 1)
    b = min(b_latency, b_overlap) if b_overlap >= granule else b_overlap
    return int(max(granule, math.ceil(b / granule) * granule))


# Nominal prior for an 8 x MI355X node over RCCL, used only when no measured fit is available (labelled as such).
# Latency ~30 us per large collective call, ~300 GB/s bus bandwidth (2 of the 7 xGMI links' worth).
NOMINAL_MI355X = {op: AlphaBeta(op, 8, 30e-6, 300e9, source="nominal prior (not measured)") for op in BUS_FACTOR}


def load_fits(path: str | None = None) -> dict[str, AlphaBeta]:
    """Fits written by ``benchmarks/comm_bench.py --fit`` (path or $DPH_COMM_FIT), else the nominal prior."""
    path = path or os.environ.get("DPH_COMM_FIT")
    if path and os.path.exists(path):
        with open(path) as fh:
            raw = json.load(fh)
        return {k: AlphaBeta(**v) for k, v in raw.items()}
    return dict(NOMINAL_MI355X)


def save_fits(fits: dict[str, AlphaBeta], path: str):
    with open(path, "w") as fh:
        json.dump({k: asdict(v) for k, v in fits.items()}, fh, indent=1)


def auto_bucket_mb(total_param_bytes: float, world: int, sharded: bool, fits: dict[str, AlphaBeta] | None = None,
                   **kw) -> float:
    """Bucket size (MiB) for the data-parallel engine: reduce-scatter buckets when sharded, all-reduce otherwise."""
    fits = fits or load_fits()
    m = fits["reduce_scatter" if sharded else "all_reduce"]
    m = AlphaBeta(m.op, world, m.alpha_s, m.beta_bus_Bps, m.source)
    return choose_bucket_bytes(m, total_param_bytes, **kw) / 2 ** 20


def measure(op: str, sizes_bytes: list[int], group=None, device=None, dtype=torch.bfloat16, iters: int = 10,
            warmup: int = 3) -> list[tuple[float, float]]:
    """Time ``op`` at each size (bytes per rank, input side) on ``group``; returns [(size, seconds)] with the
    slowest rank's time (device events on GPU, wall clock on CPU); size follows rccl-tests (all-gather: output)."""
    world = dist.get_world_size(group)
    device = device or (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
                        else torch.device("cpu"))
    esz = torch.empty((), dtype=dtype).element_size()
    out = []
    for nb in sizes_bytes:
        numel = max(world, nb // esz // world * world)
        x = torch.ones(numel, dtype=dtype, device=device)
        if op == "all_gather":
            y = torch.empty(numel * world, dtype=dtype, device=device)
            fn = lambda: dist.all_gather_into_tensor(y, x, group=group)  # noqa: E731
        elif op == "reduce_scatter":
            y = torch.empty(numel // world, dtype=dtype, device=device)
            fn = lambda: dist.reduce_scatter_tensor(y, x, group=group)  # noqa: E731
        elif op == "all_to_all":
            y = torch.empty_like(x)
            fn = lambda: dist.all_to_all_single(y, x, group=group)  # noqa: E731
        elif op == "broadcast":
            fn = lambda: dist.broadcast(x, src=dist.get_global_rank(group, 0) if group else 0, group=group)  # noqa
        else:
            fn = lambda: dist.all_reduce(x, group=group)  # noqa: E731
        for _ in range(warmup):
            fn()
        if device.type == "cuda":
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            e.synchronize()
            t = s.elapsed_time(e) / 1e3 / iters
        else:
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            t = (time.perf_counter() - t0) / iters
        tt = torch.tensor([t], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        # message size in the rccl-tests convention: all-gather counts the gathered (output) bytes
        out.append((float(numel * esz * (world if op == "all_gather" else 1)), tt.item()))
    return out


@dataclass
class StepPrediction:
    world: int
    ms_per_step: float
    exposed_comm_ms: float
    rs_ms: float
    ag_ms: float
    optimizer_ms: float
    efficiency: float        # value(N) / (N * value(1)) for a weak-scaling run


def predict_sharded_step(compute_ms: float, optimizer_ms: float, grad_bytes: float, param_bytes: float, world: int,
                         bucket_bytes: float, fits: dict[str, AlphaBeta] | None = None,
                         backward_fraction: float = 2.0 / 3.0, comm_slowdown: float = 0.0) -> StepPrediction:
    """Weak-scaling step time of the sharded data-parallel engine (parallel/data_parallel.py, shard=True: bucketed
    reduce-scatter of the gradients overlapped with backward, 1/N optimizer sweep, bucketed parameter all-gather
    overlapped with the next forward) from the 1-GPU step and the alpha-beta fits.

    ``compute_ms``: forward + backward of the 1-GPU step (its optimizer excluded: ``optimizer_ms``).  Exposed
    communication = the last reduce-scatter bucket (issued when backward ends) + the first all-gather bucket (the
    next forward waits for it) + whatever part of the reduce-scatter (all-gather) stream does not fit under the
    backward (forward) window.  ``comm_slowdown``: fractional compute slowdown while collectives run beside it
    (RCCL kernels occupy CUs); 0 unless measured.  A MODEL for planning and for checking the driver's measured
    curve against -- not a measurement."""
    if world <= 1:
        t = compute_ms + optimizer_ms
        return StepPrediction(1, t, 0.0, 0.0, 0.0, optimizer_ms, 1.0)
    fits = fits or load_fits()
    rs = AlphaBeta("reduce_scatter", world, fits["reduce_scatter"].alpha_s, fits["reduce_scatter"].beta_bus_Bps)
    ag = AlphaBeta("all_gather", world, fits["all_gather"].alpha_s, fits["all_gather"].beta_bus_Bps)
    nb_g = max(1, math.ceil(grad_bytes / bucket_bytes))
    nb_p = max(1, math.ceil(param_bytes / bucket_bytes))
    rs_ms = 1e3 * nb_g * rs.time(grad_bytes / nb_g)
    ag_ms = 1e3 * nb_p * ag.time(param_bytes / nb_p)
    bwd_ms, fwd_ms = compute_ms * backward_fraction, compute_ms * (1.0 - backward_fraction)
    exposed = 1e3 * rs.time(grad_bytes / nb_g) + 1e3 * ag.time(param_bytes / nb_p)
    exposed += max(0.0, rs_ms - bwd_ms) + max(0.0, ag_ms - fwd_ms)
    busy = compute_ms * (1.0 + comm_slowdown * min(1.0, (rs_ms + ag_ms) / compute_ms))
    t = busy + optimizer_ms / world + exposed
    t1 = compute_ms + optimizer_ms
    return StepPrediction(world, t, exposed, rs_ms, ag_ms, optimizer_ms / world, t1 / t)
