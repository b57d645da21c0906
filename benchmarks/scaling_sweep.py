#!/usr/bin/env python3
"""Weak-scaling sweep of bench.py on one node: N = 1, 2, 4, 8 ranks back to back, one rank per GPU over RCCL.

Each N runs ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py
--gpus N ...`` (N = 1 runs bench.py directly: the same sharded engine in an RCCL world of one), reads bench.py's
JSON line and reports

    tokens/s (whole job), per GPU, ms/step, and scaling efficiency E(N) = value(N) / (N * value(1))

as a Markdown table and a JSON file.  The per-GPU batch is fixed (weak scaling), so E(N) = 1 is perfect; it can
exceed 1 because N > 1 shards the optimizer state (1/N of the AdamW sweep per GPU).  This is the curve the
reference's guides discuss but never publish (BASELINE.md "Not published").

    python benchmarks/scaling_sweep.py --ns 1 2 4 8 --steps 10 --warmup 3 --out results/scaling
    python benchmarks/scaling_sweep.py --ns 1 2 -- --device cpu --model tiny --seq-len 64 --micro-batch 2
    python benchmarks/scaling_sweep.py --layouts dp tp hybrid pp resnet-fsdp --ns 1 2 4 8 --out results/all

``--layouts`` sweeps every BASELINE.json config bench.py knows (train/bench_layouts.py) under the same contract; a
layout's efficiency uses the same formula (for the strong-scaling tp layout it is speedup / N).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def bench_cmd(n: int, steps: int, warmup: int, extra: list[str]) -> list[str]:
    tail = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup)] + extra
    if n == 1:
        return [sys.executable] + tail
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + tail


def run_one(n: int, steps: int, warmup: int, extra: list[str], timeout: float, log_dir: str | None) -> dict:
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    t0 = time.perf_counter()
    p = subprocess.run(bench_cmd(n, steps, warmup, extra), capture_output=True, text=True, timeout=timeout, env=env)
    wall = time.perf_counter() - t0
    if log_dir:
        with open(os.path.join(log_dir, f"n{n}.log"), "w") as fh:
            fh.write(p.stdout + "\n---- stderr ----\n" + p.stderr)
    if p.returncode != 0:
        raise RuntimeError(f"bench.py at N={n} exited {p.returncode}:\n{p.stderr[-2000:]}")
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    if len(recs) != 1:
        raise RuntimeError(f"bench.py at N={n} printed {len(recs)} result lines")
    rec = recs[0]
    rec["wall_s"] = round(wall, 1)
    return rec


def efficiency_table(recs: dict[int, dict]) -> tuple[list[dict], str]:
    base = recs.get(1)
    rows = []
    for n in sorted(recs):
        r = recs[n]
        eff = r["value"] / (n * base["value"]) if base else None
        rows.append({"n_gpus": n, "value": r["value"], "unit": r["unit"], "tokens_per_s": r["value"],
                     "tokens_per_s_per_gpu": round(r["value"] / n, 1),
                     "ms_per_step": r["ms_per_step"], "parallelism": r["config"]["parallelism"],
                     "global_batch": r["config"]["global_batch"], "peak_hbm_gb": r.get("peak_hbm_gb"),
                     "scaling_efficiency": None if eff is None else round(eff, 4)})
    unit = next(iter(recs.values()))["unit"] if recs else "tokens/s"
    lines = [f"| N | parallelism | global batch | {unit} | per GPU | ms/step | efficiency |",
             "|---|---|---|---|---|---|---|"]
    for row in rows:
        e = "—" if row["scaling_efficiency"] is None else f"{100 * row['scaling_efficiency']:.1f} %"
        lines.append(f"| {row['n_gpus']} | {row['parallelism']} | {row['global_batch']} | {row['tokens_per_s']:,.0f} "
                     f"| {row['tokens_per_s_per_gpu']:,.0f} | {row['ms_per_step']:.1f} | {e} |")
    return rows, "\n".join(lines)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    extra: list[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=900.0, help="seconds per N")
    ap.add_argument("--out", default=None, help="directory for n<N>.log, scaling.json and scaling.md")
    ap.add_argument("--layouts", nargs="+", default=None,
                    help="sweep these bench.py layouts (dp tp hybrid pp resnet-fsdp), one sub-directory of --out each")
    args = ap.parse_args(argv)
    if args.layouts:
        out = {}
        for lay in args.layouts:
            sub = ["--ns", *map(str, args.ns), "--steps", str(args.steps), "--warmup", str(args.warmup),
                   "--timeout", str(args.timeout)]
            if args.out:
                sub += ["--out", os.path.join(args.out, lay)]
            print(f"[scaling] layout {lay}", flush=True)
            out[lay] = main(sub + ["--"] + extra + ["--layout", lay])
        return out
    if args.out:
        os.makedirs(args.out, exist_ok=True)
    recs: dict[int, dict] = {}
    for n in args.ns:
        recs[n] = run_one(n, args.steps, args.warmup, extra, args.timeout, args.out)
        print(f"[scaling] N={n}: {recs[n]['value']:,.1f} {recs[n]['unit']} ({recs[n]['ms_per_step']:.1f} ms/step)",
              flush=True)
    rows, md = efficiency_table(recs)
    print(md)
    if args.out:
        with open(os.path.join(args.out, "scaling.json"), "w") as fh:
            json.dump({"metric": next(iter(recs.values()))["metric"], "rows": rows, "bench_args": extra,
                       "steps": args.steps, "warmup": args.warmup}, fh, indent=1)
        with open(os.path.join(args.out, "scaling.md"), "w") as fh:
            fh.write(md + "\n")
    return rows


if __name__ == "__main__":
    main()
