#!/usr/bin/env python3
"""Launch a configs/*.yaml workload: one rank per GPU on this node via torch.distributed.run (RCCL), or the
single-process path for nproc_per_node == 1.

    python scripts/run_config.py configs/llama2_7b_fsdp2_tp4.yaml [--nproc N] [--dry-run] [-- extra driver args]

YAML keys: ``driver`` (path relative to the repo root), ``nproc_per_node``, ``args`` (flag -> value; ``true``
emits a bare flag, ``false`` omits it).  Extra arguments after ``--`` are appended (later flags win).
"""
from __future__ import annotations

import argparse
import os
import shlex
import socket
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def to_argv(args: dict) -> list[str]:
    out = []
    for k, v in (args or {}).items():
        if v is True:
            out.append(f"--{k}")
        elif v is False or v is None:
            continue
        else:
            out += [f"--{k}", str(v)]
    return out


def build_command(cfg: dict, nproc: int | None = None, extra: list[str] | None = None, port: int | None = None):
    n = int(nproc or cfg.get("nproc_per_node", 1))
    driver = os.path.join(ROOT, cfg["driver"])
    argv = to_argv(cfg.get("args")) + list(extra or [])
    if n == 1:
        return [sys.executable, driver] + argv
    if port is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), driver] + argv


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("config")
    ap.add_argument("--nproc", type=int, default=None)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    with open(a.config) as fh:
        cfg = yaml.safe_load(fh)
    cmd = build_command(cfg, a.nproc, extra)
    print("+ " + " ".join(shlex.quote(c) for c in cmd), flush=True)
    if a.dry_run:
        return 0
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    n = int(a.nproc or cfg.get("nproc_per_node", 1))
    if str((cfg.get("args") or {}).get("device", "")) == "cpu" and "OMP_NUM_THREADS" not in env:
        # CPU ranks split the node's cores (torchrun would default every rank to 1 thread, a bare launch to all
        # cores): ResNet-50 DDP/gloo on 8 cores, 2 ranks -- 1 thread 5.6 img/s, 8 threads 3.4, 4 threads 16.8
        try:
            cores = len(os.sched_getaffinity(0))
        except AttributeError:
            cores = os.cpu_count() or 1
        env["OMP_NUM_THREADS"] = str(max(1, cores // n))
    return subprocess.call(cmd, env=env, cwd=ROOT)


if __name__ == "__main__":
    sys.exit(main())
