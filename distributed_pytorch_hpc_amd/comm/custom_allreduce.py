"""Single-node all-reduce over IPC-mapped peer buffers (csrc/custom_allreduce.hip).

The reference leaves every all-reduce to NCCL rings (DDP buckets, C1; Rowwise TP outputs, C11 -- SURVEY.md
§2.12).  On an MI355X node the 8 GPUs are a full xGMI mesh, so a small or medium all-reduce is faster when every
rank reads its peers' buffers directly over all 7 links at once:

* one-shot (<= 256 KiB or 2 ranks): each rank reduces the whole message from all peers -- one barrier;
* two-shot: reduce-scatter by direct peer reads, then all-gather by direct peer reads -- two barriers.

Results are bit-identical on every rank (fp32 accumulation in rank order).  The staging buffers are registered
once (``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle``; handles exchanged with one ``all_gather_object``), so a
call costs one kernel launch and can be captured in a HIP graph.

Use::

    car = XgmiAllReduce(group)            # collective: every rank of the group constructs it
    car.all_reduce(t)                     # in place, SUM (op="avg" divides by the group size)

``get_custom_allreduce(group)`` returns a cached instance, or ``None`` when the group is not eligible (CPU/gloo,
more than 8 ranks, ranks on several hosts, native extension missing).

Which path a message takes is decided from data (reference: the timing loop of tests/torch_comm_bench.py:62-116):
``probe_crossover(group)`` times RCCL's all-reduce and this one at 4 KiB .. 16 MiB on the job's own group (slowest
rank's time, so every rank decides alike), and ``choose_crossover`` turns the samples into the largest message
size up to which the direct-peer path wins at every measured size (0 when RCCL wins already at the smallest).
``set_policy(group, crossover)`` records it; ``comm.functional.all_reduce_`` -- which the TP row-parallel
all-reduce, the sequence-parallel norm-gradient reduction and the loss-parallel reductions go through -- and the
data-parallel engine's buckets then route SUM messages up to the crossover here.  ``DPH_CUSTOM_ALLREDUCE=1`` forces
the path up to ``DPH_CUSTOM_ALLREDUCE_MAX_BYTES`` (8 MiB), ``=0`` disables it; unset = the measured policy (none
recorded: RCCL).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib

_ALGOS = {"auto": 0, "oneshot": 1, "twoshot": 2}
_MAX_RANKS = 8


def _group_ranks(group):
    return dist.get_world_size(group), dist.get_rank(group)


class XgmiAllReduce:
    def __init__(self, group=None, max_bytes: int = 64 << 20, timeout_s: float = None, max_blocks: int = 64):
        timeout_s = _TIMEOUT_S if timeout_s is None else timeout_s
        if not dist.is_initialized():
            raise RuntimeError("XgmiAllReduce needs an initialised process group")
        _lib.require()
        self.group = group
        self.world, self.rank = _group_ranks(group)
        if self.world > _MAX_RANKS:
            raise ValueError(f"XgmiAllReduce supports at most {_MAX_RANKS} ranks (got {self.world})")
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise ValueError("XgmiAllReduce: all ranks of the group must be on one node")
        self.max_bytes = int(max_bytes)
        self.max_blocks = int(max_blocks)
        ops = _lib.ops()
        self._ops = ops
        self.ctx = ops.car_create(self.rank, self.world, self.max_bytes, float(timeout_s))
        mine = ops.car_ipc_handle(self.ctx)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(mine.numpy().tobytes()), group=group)
        table = torch.tensor([list(h) for h in handles], dtype=torch.uint8)
        ops.car_open(self.ctx, table.contiguous())
        dist.barrier(group=group)
        self._flag = None           # int32 [1] device scratch of the step guard (guard_update)
        self._guard_event = None    # event after the last guard: its verdict is readable once it completes

    # ------------------------------------------------------------------------------------------------
    def supports(self, t: torch.Tensor) -> bool:
        """Rank-invariant eligibility (shape / dtype / layout only), so every rank takes the same path."""
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and nbytes % 16 == 0 and 0 < nbytes <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor, op: str = "sum", out: Optional[torch.Tensor] = None,
                   algo: str = "auto") -> torch.Tensor:
        """All-reduce ``t`` (in place unless ``out`` is given) and return the result tensor."""
        if not self.supports(t):
            raise ValueError("XgmiAllReduce: tensor must be a contiguous 16-B aligned bf16/fp32 GPU tensor of at most "
                             f"{self.max_bytes} bytes (multiple of 16)")
        if op not in ("sum", "avg"):
            raise ValueError("op must be 'sum' or 'avg'")
        out = t if out is None else out
        scale = 1.0 / self.world if op == "avg" else 1.0
        src = t if t.data_ptr() % 16 == 0 else t.clone()
        dst = out if out.data_ptr() % 16 == 0 else torch.empty_like(out)
        self._ops.car_allreduce(self.ctx, src, dst, _ALGOS[algo], scale, self.max_blocks)
        if dst is not out:
            out.copy_(dst)
        return out

    def errors(self) -> int:
        """Non-zero once a barrier of this rank's kernels timed out (0 when healthy).  No device synchronisation:
        the kernel writes a host-mapped word, so a kernel still in flight reports on a later call."""
        return int(self._ops.car_status(self.ctx))

    def agreed_error(self) -> int:
        """The group-agreed verdict written by the last ``guard_update`` (non-zero: some rank's barrier timed out).
        Authoritative once that guard's event has completed."""
        return int(self._ops.car_agreed(self.ctx))

    def close(self):
        if getattr(self, "ctx", None):
            self._ops.car_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_CACHE: dict = {}


_POLICY: dict = {}        # group key -> crossover bytes (messages <= it take the direct-peer path)
_ANY_BACKEND: set = set()  # group keys allowed on a non-RCCL group (tests: gloo ranks sharing one GPU)


def _key(group):
    return id(group) if group is not None else "world"


def custom_allreduce_enabled() -> bool:
    return os.environ.get("DPH_CUSTOM_ALLREDUCE", "0") == "1"


def custom_allreduce_max_bytes() -> int:
    return int(os.environ.get("DPH_CUSTOM_ALLREDUCE_MAX_BYTES", str(8 << 20)))


def set_policy(group, crossover_bytes: int, allow_any_backend: bool = False) -> None:
    """Record the measured crossover for ``group`` (0 = always RCCL).  ``allow_any_backend``: also on a non-RCCL
    group whose tensors live on GPUs (processes sharing one GPU in tests)."""
    _POLICY[_key(group)] = int(crossover_bytes)
    if allow_any_backend:
        _ANY_BACKEND.add(_key(group))


def clear_policy(group=None) -> None:
    _POLICY.pop(_key(group), None)
    _ANY_BACKEND.discard(_key(group))


_DEAD: set = set()        # group keys whose direct-peer path failed its health check: never used again


def policy_max_bytes(group) -> int:
    """Largest message (bytes) the direct-peer path takes on ``group``: 0 once the group's path failed a health check
    (whatever the environment says), else the env override, else the measured crossover, else 0."""
    if _key(group) in _DEAD:
        return 0
    env = os.environ.get("DPH_CUSTOM_ALLREDUCE")
    if env == "1":
        return custom_allreduce_max_bytes()
    if env == "0":
        return 0
    return _POLICY.get(_key(group), 0)


def use_custom(t: torch.Tensor, group) -> Optional["XgmiAllReduce"]:
    """The XgmiAllReduce to run this SUM all-reduce on, or None for RCCL.  Rank-invariant: the decision depends on
    the message size, the recorded policy and the group only."""
    limit = policy_max_bytes(group)
    if limit <= 0 or not t.is_cuda or t.numel() * t.element_size() > limit:
        return None
    car = get_custom_allreduce(group)
    return car if car is not None and car.supports(t) else None


def choose_crossover(samples: list) -> int:
    """samples: [(bytes, t_rccl_s, t_xgmi_s)] -> the largest size up to which the direct-peer path is faster at EVERY
    measured size (sizes above the first loss go to RCCL), 0 if RCCL wins at the smallest size."""
    best = 0
    for nbytes, t_rccl, t_xgmi in sorted(samples):
        if t_xgmi is None or not (t_xgmi < t_rccl):
            break
        best = int(nbytes)
    return best


def probe_crossover(group=None, sizes=(4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20),
                    iters: int = 10, warmup: int = 3, dtype=torch.bfloat16) -> dict:
    """Time RCCL's all-reduce and the direct-peer one on ``group`` at ``sizes`` bytes; every rank gets the same
    (max over ranks) times and the same crossover.  Collective.  Returns {"samples": [...], "crossover_bytes": n}."""
    car = get_custom_allreduce(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    world = dist.get_world_size(group)
    samples = []
    ok = torch.ones(1, dtype=torch.float64, device=dev)
    for nbytes in sizes:
        n = max(8, nbytes // torch.empty((), dtype=dtype).element_size())
        x = torch.ones(n, dtype=dtype, device=dev)
        times = []
        for path in ("rccl", "xgmi"):
            if path == "xgmi" and (car is None or not car.supports(x)):
                times.append(None)
                continue

            def run():
                if path == "rccl":
                    dist.all_reduce(x, group=group)
                else:
                    car.all_reduce(x)

            for _ in range(warmup):
                run()
            torch.cuda.synchronize(dev)
            dist.barrier(group=group)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                x.fill_(1.0)
                run()
            e.record()
            e.synchronize()
            if path == "xgmi" and not (torch.all(x == world) and car.errors() == 0):
                ok.zero_()      # wrong sums or barrier timeouts: never route traffic to this path
            x.fill_(1.0)
            t = torch.tensor([s.elapsed_time(e) / iters / 1e3], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            times.append(float(t.item()))
        samples.append((int(nbytes), times[0], times[1]))
    # whether the xgmi arm exists is itself rank-invariant (every rank constructs or fails alike); correctness is
    # agreed on (MIN over ranks) so a path that failed anywhere is off everywhere
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    verified = bool(ok.item() == 1.0)
    if not verified:
        drop(group)
    return {"samples": samples, "verified": verified,
            "crossover_bytes": choose_crossover(samples) if verified else 0}


def active() -> bool:
    """True when some group has a live direct-peer instance (the engines then run ``guard_update`` every step)."""
    return any(car is not None for car in _CACHE.values())


def guard_update(gscale: torch.Tensor) -> None:
    """Stream-ordered health guard: call between a step's last reduction and its optimizer kernels, on the stream
    that runs them, with the step's device gradient scale.  For every live direct-peer instance (in cache order,
    which is the same on every rank: instances are created collectively) it copies this rank's barrier-timeout word
    to the device, MAX-all-reduces it over the instance's group through the process-group backend (never through the
    possibly broken path itself) and, if any rank of the group timed out, sets ``gscale`` to NaN -- the optimizer
    kernels then skip the update on every rank of the group alike -- and records the agreed verdict for
    ``check_health``.  Every rank of every such group must call it (the engines do, once per step).
    Advisor r5: the host-side check alone ran before the update kernels were queued, so the update of the step whose
    all-reduce timed out still ran on its sums; and the per-rank word let only the waiting ranks disable the path."""
    for car in list(_CACHE.values()):
        if car is None:
            continue
        if car._flag is None or car._flag.device != gscale.device:
            car._flag = torch.zeros(1, dtype=torch.int32, device=gscale.device)
        car._ops.car_flag(car.ctx, car._flag)
        dist.all_reduce(car._flag, op=dist.ReduceOp.MAX, group=car.group)
        car._ops.car_poison(car.ctx, car._flag, gscale)
        ev = torch.cuda.Event()
        ev.record()
        car._guard_event = ev


def drop(group=None) -> None:
    """Forget ``group``'s direct-peer instance (after a failed probe; every rank calls it alike): nothing is ever
    routed to it again, and a barrier timeout it recorded does not surface later as a training-step
    XgmiAllReduceError (check_health)."""
    key = _key(group)
    car = _CACHE.get(key)
    _CACHE[key] = None
    _POLICY.pop(key, None)
    if car is not None:
        car.close()


class XgmiAllReduceError(RuntimeError):
    """A direct-peer all-reduce barrier timed out: its sums may hold a peer's stale staging data."""


def check_health() -> None:
    """Raise XgmiAllReduceError if a direct-peer all-reduce barrier timed out, after turning the path off for that
    group for good (``_DEAD``: RCCL takes every later message, ``DPH_CUSTOM_ALLREDUCE=1`` included).

    A timed-out barrier lets the kernel finish with whatever the late peer's staging buffer held.  The update that
    would consume such sums is already skipped on the device by ``guard_update`` (same step, every rank of the group);
    this host check reports it.  It reads the group-agreed verdict of the previous step's guard after that guard's
    event (in steady state it completed long ago: the host is at most one step ahead), so every rank raises at the
    same step and drops the same groups -- a caller that catches the error keeps routing identically on every rank.
    The timeout of the current step's reductions is reported at the next step.  An instance that never ran a guard
    (direct use, inference) falls back to this rank's own timeout word."""
    bad = []
    for key, car in list(_CACHE.items()):
        if car is None:
            continue
        if car._guard_event is not None:
            car._guard_event.synchronize()
            failed = car.agreed_error()
        else:
            failed = car.errors()
        if failed:
            bad.append(key)
    for key in bad:
        _DEAD.add(key)
        _POLICY.pop(key, None)
        car = _CACHE.get(key)
        _CACHE[key] = None
        if car is not None:
            car.close()
    if bad:
        raise XgmiAllReduceError(
            f"direct-peer xGMI all-reduce barrier timed out on {len(bad)} group(s) (a peer stalled > "
            f"{_TIMEOUT_S:.0f} s); the optimizer update that would have used those sums was skipped on every rank of "
            "the group, and the path is now disabled for those groups.")


_TIMEOUT_S = 10.0


def get_custom_allreduce(group=None) -> Optional[XgmiAllReduce]:
    """Cached XgmiAllReduce for ``group`` or None if the group cannot use it (collective on first call)."""
    if not dist.is_initialized():
        return None
    if dist.get_backend(group) != "nccl" and _key(group) not in _ANY_BACKEND:
        return None
    key = _key(group)
    if key in _DEAD:
        return None
    if key not in _CACHE:
        try:
            # staging sized for the probe's largest message (16 MiB) or a larger forced / recorded limit
            _CACHE[key] = XgmiAllReduce(group, max_bytes=max(custom_allreduce_max_bytes(), _POLICY.get(key, 0),
                                                             16 << 20))
        except (ValueError, RuntimeError):
            _CACHE[key] = None
    return _CACHE[key]
