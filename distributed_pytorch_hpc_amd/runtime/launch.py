"""Single-node multi-rank launcher with a gang watchdog and restart-from-checkpoint.

Replaces the reference's PBS + ``mpiexec -n N --ppn 4`` / ``mpiexec ... torchrun`` job templates
(scripts/**/run_*.sh, scripts/torchrun_multigpu_pbs.sh:152, SURVEY.md L-PBS / L-TR) for one 8-GPU MI355X node:

    python -m distributed_pytorch_hpc_amd.runtime.launch --nproc 8 [--log-dir logs] [--max-restarts 2] \
        [--timeout 3600] [--backend nccl|gloo] train.py --args ...

Each rank gets the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1,
MASTER_PORT) plus DPH_LAUNCHER=dph and DPH_RESTART_COUNT.  The watchdog polls the gang: the first
rank that exits non-zero (or a --timeout) tears the whole gang down (SIGTERM to every rank's process group, SIGKILL
after a grace period) -- no rank is left blocked in a collective -- and, while restarts remain, relaunches on a
fresh port; training scripts resume from their latest checkpoint (utils.checkpointing.ShardedCheckpointer).
``--log-dir`` writes rank{r}.out / rank{r}.err per rank (utils/redirect.py semantics at the process level).
``--cpu-bind numa`` (default) pins each rank to its share of the cores local to its GPU's NUMA node
(runtime/device.py; set in the child before it execs Python, so before any GPU call) and sizes OMP_NUM_THREADS
to that share; ``--cpu-bind none`` reproduces the reference's unbound ranks (run_fsdp.sh:64).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

from . import device
from .env import free_port


def _bind(cpus):
    """preexec_fn: runs in the forked child before exec -- pins the rank's CPU set (no GPU state exists yet)."""
    def fn():
        if cpus:
            os.sched_setaffinity(0, cpus)
    return fn


def bindings(args):
    if getattr(args, "cpu_bind", "numa") != "numa":
        return None
    return device.plan(args.nproc, omp_threads=args.omp_threads)


def _spawn(args, attempt: int, port: int):
    procs = []
    binds = bindings(args)
    if binds and attempt == 0:
        print("[dph.launch] CPU binding:\n" + device.describe(binds), file=sys.stderr, flush=True)
    for r in range(args.nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.nproc), LOCAL_WORLD_SIZE=str(args.nproc),
                   GROUP_RANK="0", MASTER_ADDR=args.master_addr, MASTER_PORT=str(port), DPH_LAUNCHER="dph",
                   DPH_RESTART_COUNT=str(attempt))
        if args.backend:
            env["DPH_BACKEND"] = args.backend
        b = binds[r] if binds else None
        if b is not None:
            env["DPH_CPU_BIND"] = ",".join(map(str, b.cpus)) if b.cpus else "none"
            env["DPH_NUMA_NODE"] = str(b.numa_node)
        if args.omp_threads:
            env["OMP_NUM_THREADS"] = str(args.omp_threads)
        elif b is not None and b.cpus and "OMP_NUM_THREADS" not in os.environ:
            env["OMP_NUM_THREADS"] = str(b.omp_threads)
        elif "OMP_NUM_THREADS" not in env:   # ranks split the cores instead of oversubscribing them
            try:
                cores = len(os.sched_getaffinity(0))
            except AttributeError:
                cores = os.cpu_count() or 1
            env["OMP_NUM_THREADS"] = str(max(1, cores // max(args.nproc, 1)))
        out = err = None
        if args.log_dir:
            os.makedirs(args.log_dir, exist_ok=True)
            out = open(os.path.join(args.log_dir, f"rank{r}.out"), "a")
            err = open(os.path.join(args.log_dir, f"rank{r}.err"), "a")
        cmd = [sys.executable, "-u", args.script] + args.script_args
        p = subprocess.Popen(cmd, env=env, stdout=out, stderr=err, start_new_session=True,
                             preexec_fn=_bind(b.cpus) if b is not None and b.cpus else None)
        procs.append((p, out, err))
    return procs


def _kill_all(procs, grace: float):
    for p, _, _ in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p, _, _ in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run(args) -> int:
    attempt = 0
    while True:
        port = args.master_port if (args.master_port and attempt == 0) else free_port()
        procs = _spawn(args, attempt, port)
        t0 = time.time()
        failed_rank, code = None, 0
        while True:
            codes = [p.poll() for p, _, _ in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed_rank, code = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if args.timeout and time.time() - t0 > args.timeout:
                failed_rank, code = -1, 124
                break
            time.sleep(0.1)
        if failed_rank is not None:
            what = "timeout" if failed_rank == -1 else f"rank {failed_rank} exited with {code}"
            print(f"[dph.launch] attempt {attempt}: {what}; stopping the gang", file=sys.stderr, flush=True)
            _kill_all(procs, args.grace)
        for _, o, e in procs:
            for f in (o, e):
                if f:
                    f.close()
        if failed_rank is None:
            return 0
        if attempt >= args.max_restarts:
            return code if code else 1
        attempt += 1
        print(f"[dph.launch] restarting (attempt {attempt}/{args.max_restarts})", file=sys.stderr, flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", "--nproc-per-node", dest="nproc", type=int, default=8)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--backend", default=None, help="exported as DPH_BACKEND for the training script")
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=0.0, help="seconds; 0 = none")
    ap.add_argument("--grace", type=float, default=10.0)
    ap.add_argument("--omp-threads", type=int, default=0)
    ap.add_argument("--cpu-bind", choices=["numa", "none"], default="numa",
                    help="numa: pin each rank to its share of its GPU's NUMA-local cores; none: no binding")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    sys.exit(run(args))


if __name__ == "__main__":
    main()
