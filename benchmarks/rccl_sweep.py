#!/usr/bin/env python3
"""RCCL environment-knob sweep on one node: run ``comm_bench.py`` once per environment variant (channels, protocol,
algorithm, MSCCL / MSCCL++) and pick, per collective and message size, the variant with the highest bus bandwidth.

The reference's tuning advice is a fixed block of NCCL / Slingshot exports (README.md:198-210,
docs/guide/nccl_tuning.md) that was never measured; on an xGMI node none of its fabric knobs apply and what matters
is RCCL's channel count and protocol per message size.  This driver turns ``docs/guide/rccl_tuning.md``'s knob table
into data: every variant runs in its own ``torch.distributed.run`` job (RCCL reads its environment once, at
communicator creation), the per-variant JSON files are kept, and the summary names

  * the winning variant per (op, size) and its speed-up over RCCL's defaults;
  * one recommended variant for the framework's own traffic -- the geometric mean of its busbw ratio to the
    defaults over the reduce-scatter / all-gather sizes of the data-parallel buckets (32-512 MiB), where the bench's time goes, and at
    least --min-gain (3 %) above them -- written as an ``export`` file that ``scripts/env_mi355x.sh`` users can source.

    python benchmarks/rccl_sweep.py --nproc 8 --out results/rccl_sweep           # 8 x MI355X
    python benchmarks/rccl_sweep.py --nproc 2 --backend gloo --variants base,ch32 --sizes 1e3,1e4 --out /tmp/s
      (gloo ignores the RCCL knobs: CPU rehearsal of the driver only)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> environment overrides (empty = RCCL's own topology-aware defaults)
VARIANTS: dict[str, dict[str, str]] = {
    "base": {},
    "ch16": {"NCCL_MIN_NCHANNELS": "16"},
    "ch32": {"NCCL_MIN_NCHANNELS": "32"},
    "ch64": {"NCCL_MIN_NCHANNELS": "64", "NCCL_MAX_NCHANNELS": "64"},
    "simple": {"NCCL_PROTO": "Simple"},
    "ll128": {"NCCL_PROTO": "LL128"},
    "ring": {"NCCL_ALGO": "Ring"},
    "tree": {"NCCL_ALGO": "Tree"},
    "msccl_off": {"RCCL_MSCCL_ENABLE": "0"},
    "mscclpp": {"RCCL_MSCCLPP_ENABLE": "1"},
}
# message sizes (elements per rank, bf16): 2 KB ... 512 MiB; the top three are data-parallel bucket sizes
DEFAULT_SIZES = "1e3,1e4,1e5,1e6,4e6,1.6e7,6.7e7,1.34e8,2.68e8"
BUCKET_BYTES = (32 << 20, 512 << 20)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_variant(name: str, over: dict, args, out_dir: str) -> dict:
    path = os.path.join(out_dir, f"{name}.json")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "benchmarks", "comm_bench.py"), "--ops", args.ops, "--sizes", args.sizes,
           "--dtype", args.dtype, "--iters", str(args.iters), "--warmup", str(args.warmup), "--json", path]
    if args.backend:
        cmd += ["--backend", args.backend]
    env = {k: v for k, v in os.environ.items() if not k.startswith(("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCH",
                                                                     "NCCL_MAX_NCH", "RCCL_MSCCL"))}
    env.update(over, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout, env=env)
    with open(os.path.join(out_dir, f"{name}.log"), "w") as fh:
        fh.write(" ".join(f"{k}={v}" for k, v in over.items()) + "\n" + p.stdout + "\n---- stderr ----\n" + p.stderr)
    if p.returncode != 0 or not os.path.exists(path):
        return {"name": name, "env": over, "ok": False, "rc": p.returncode, "stderr": p.stderr[-800:]}
    with open(path) as fh:
        res = json.load(fh)["results"]
    return {"name": name, "env": over, "ok": True, "wall_s": round(time.perf_counter() - t0, 1), "results": res}


def summarise(runs: list[dict], min_gain: float = 1.03) -> dict:
    """Per (op, bytes): best variant and its busbw vs base; one recommended variant for the bucket-sized
    reduce-scatter / all-gather traffic (geometric mean of busbw ratios vs base); a variant has to beat the defaults by
    ``min_gain`` to be recommended."""
    ok = [r for r in runs if r["ok"]]
    table: dict[tuple, dict] = {}
    for r in ok:
        for row in r["results"]:
            table.setdefault((row["op"], row["bytes"]), {})[r["name"]] = row["busbw_GBps"]
    best = []
    for (op, nbytes), per in sorted(table.items()):
        name = max(per, key=per.get)
        base = per.get("base")
        best.append({"op": op, "bytes": nbytes, "best": name, "busbw_GBps": round(per[name], 2),
                     "base_busbw_GBps": round(base, 2) if base else None,
                     "speedup_vs_base": round(per[name] / base, 3) if base else None})
    score = {}
    for r in ok:
        ratios = [per[r["name"]] / per["base"] for (op, nb), per in table.items()
                  if op in ("reduce_scatter", "all_gather") and BUCKET_BYTES[0] <= nb <= BUCKET_BYTES[1]
                  and "base" in per and r["name"] in per and per["base"] > 0]
        if ratios:
            score[r["name"]] = math.exp(sum(math.log(max(x, 1e-9)) for x in ratios) / len(ratios))
    rec = max(score, key=score.get) if score else None
    if rec is not None and score[rec] < min_gain:
        rec = "base"   # within run-to-run noise of RCCL's defaults: recommend nothing
    return {"best_per_size": best, "bucket_traffic_score_vs_base": {k: round(v, 4) for k, v in score.items()},
            "recommended": rec, "failed": [{"name": r["name"], "rc": r["rc"]} for r in runs if not r["ok"]]}


def write_env_file(out: str, rec, nproc: int, scores: dict, backend=None) -> str | None:
    """Write ``rccl_env.sh`` for the recommended variant, or remove a stale one.  A gloo rehearsal measures noise (gloo
    ignores every RCCL knob) and a sweep without a winner ("base" or none) must not leave an older recommendation for
    scripts/env_mi355x.sh to pick up.  Each export only fills a knob the user left unset, and the file records the
    rank count it was measured at (env_mi355x.sh skips it for another)."""
    env_path = os.path.join(out, "rccl_env.sh")
    if backend == "gloo" or rec in (None, "base") or not VARIANTS.get(rec):
        if os.path.exists(env_path):
            os.remove(env_path)
        why = "gloo rehearsal" if backend == "gloo" else "no variant beat RCCL's defaults"
        print(f"[sweep] no export file written ({why})")
        return None
    with open(env_path, "w") as fh:
        fh.write(f"# benchmarks/rccl_sweep.py: best variant for 32-512 MiB reduce-scatter / all-gather on "
                 f"{nproc} ranks (x{scores.get(rec, float('nan')):.3f} vs RCCL defaults)\n")
        fh.write(f"DPH_RCCL_SWEEP_NPROC={nproc}\n")
        for k, v in VARIANTS[rec].items():
            fh.write(f": ${{{k}:={v}}}; export {k}\n")
    print(f"[sweep] recommended for bucket traffic: {rec} {VARIANTS[rec]} -> {env_path}")
    return env_path


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", type=int, default=8)
    ap.add_argument("--variants", default=",".join(VARIANTS), help="comma list of " + ", ".join(VARIANTS))
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--sizes", default=DEFAULT_SIZES, help="elements per rank (comma list)")
    ap.add_argument("--dtype", default="bfloat16", choices=["float32", "bfloat16"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--backend", default=None, help="gloo: CPU rehearsal (knobs have no effect)")
    ap.add_argument("--timeout", type=float, default=600.0, help="seconds per variant")
    ap.add_argument("--min-gain", type=float, default=1.03, help="recommend a knob only above this speed-up")
    ap.add_argument("--out", default="results/rccl_sweep")
    args = ap.parse_args(argv)
    os.makedirs(args.out, exist_ok=True)
    names = [v for v in args.variants.split(",") if v]
    unknown = [v for v in names if v not in VARIANTS]
    if unknown:
        ap.error(f"unknown variants {unknown}")
    if "base" not in names:
        names.insert(0, "base")   # every speed-up is relative to RCCL's defaults
    runs = []
    for name in names:
        r = run_variant(name, VARIANTS[name], args, args.out)
        print(f"[sweep] {name:10s} {'ok' if r['ok'] else 'FAILED rc=%s' % r['rc']}", flush=True)
        runs.append(r)
    summ = summarise(runs, args.min_gain)
    summ["nproc"], summ["dtype"], summ["variants"] = args.nproc, args.dtype, {n: VARIANTS[n] for n in names}
    with open(os.path.join(args.out, "summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    for row in summ["best_per_size"]:
        print(f"{row['op']:15s} {row['bytes'] / 2 ** 20:10.3f} MiB  best {row['best']:10s} "
              f"{row['busbw_GBps']:8.2f} GB/s  (base {row['base_busbw_GBps']}, x{row['speedup_vs_base']})")
    write_env_file(args.out, summ["recommended"], args.nproc, summ.get("bucket_traffic_score_vs_base", {}),
                   args.backend)
    return summ


if __name__ == "__main__":
    main()
