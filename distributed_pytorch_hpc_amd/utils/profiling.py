"""Profiling: torch.profiler wrapper, roctx ranges, and a rocprofv3 command builder.

Capability parity with utils/profiling.py:25-86 of the reference (``training_profiler`` context manager with a
wait/warmup/active schedule and TensorBoard/Chrome traces, ``print_profiler_summary``), plus:
  * traces are written for EVERY rank (comm skew between ranks is the thing to look for), not rank 0 only;
  * ``range(name)`` emits a roctx range (visible in rocprofv3 --marker-trace and in torch.profiler) around
    step phases (forward / backward / optimizer / comm);
  * ``rocprof_cmd`` builds the kernel-trace / counter command lines used for the profiles/ evidence
    (``rocprofv3 --kernel-trace --stats``; counters in a separate run, never with --sys-trace).
"""
from __future__ import annotations

import contextlib
import os
from typing import Iterable, Optional

import torch


@contextlib.contextmanager
def training_profiler(output_dir: str = "profiler_output", wait: int = 1, warmup: int = 1, active: int = 3,
                      repeat: int = 1, rank: Optional[int] = None, record_shapes: bool = True,
                      profile_memory: bool = True, with_stack: bool = False, all_ranks: bool = True):
    """Yields a torch.profiler.profile; the caller must call ``prof.step()`` once per iteration."""
    from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler

    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)  # HIP kernels via roctracer on ROCm
    handler = None
    if all_ranks or rank == 0:
        os.makedirs(output_dir, exist_ok=True)
        handler = tensorboard_trace_handler(output_dir, worker_name=f"rank{rank}")
    with profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active, repeat=repeat),
                 on_trace_ready=handler, record_shapes=record_shapes, profile_memory=profile_memory,
                 with_stack=with_stack) as prof:
        yield prof


def print_profiler_summary(prof, rank: int = 0, top_n: int = 20, sort_by: str = "cuda_time_total") -> str:
    if rank != 0:
        return ""
    try:
        table = prof.key_averages().table(sort_by=sort_by, row_limit=top_n)
    except Exception:
        table = prof.key_averages().table(sort_by="cpu_time_total", row_limit=top_n)
    print(table)
    return table


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    """roctx range (torch.cuda.nvtx maps to roctx on ROCm builds); no-op without a GPU."""
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:
            pushed = False
    with torch.autograd.profiler.record_function(name):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


def rocprof_cmd(argv: Iterable[str], out_dir: str = "gpurun_out/prof", stats: bool = True,
                counters: Optional[list[str]] = None) -> list[str]:
    """rocprofv3 command for ``argv`` (program FIRST after ``--``, no env/bash hops)."""
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", out_dir, "-o", "run"]
    if stats:
        cmd.append("--stats")
    if counters:
        cmd += ["--pmc", " ".join(counters)]
    return cmd + ["--"] + list(argv)


def summarize_kernel_stats(csv_path: str, top: int = 25) -> list[dict]:
    """Top kernels of a rocprofv3 *_kernel_stats.csv (name, calls, total ms, share)."""
    import csv

    rows = list(csv.DictReader(open(csv_path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    return [{"name": r["Name"][:140], "calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
             "pct": float(r["Percentage"])} for r in rows[:top]]
