#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel and per-category GPU time.

Reads either rocprofv3's SQLite output (``<dir>/<name>_results.db``, the default format) or its CSV
kernel trace (``--output-format csv`` -> ``*_kernel_trace.csv``).  Optionally restricts to the last
``--last-ms`` of GPU activity (the timed steps of a bench run) and divides by ``--steps``.

A time window mis-counts steps when tracing slows a host-bound step down (an eager SimpleUNet step runs ~25 % longer
under rocprofv3, so "the last 4 x ms_per_step" held about 3 steps and every per-step figure read 25 % low).
``--step-marker NAME --run-steps N`` counts steps instead: the marker kernel's launches per step are its total count
over the N steps the traced run executed, and the window is the last ``--steps`` steps' worth of its launches.
``--step-ms`` (the un-traced bench's ms/step) adds ``idle_vs_step_pct`` = 1 - kernel busy / step time, the host gap
share of the real step rather than of the traced one.

    python benchmarks/prof_summary.py gpurun_out/prof3 --steps 2 --json profiles/x.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sqlite3
from collections import defaultdict

CATEGORIES = [
    ("conv(miopen/ck)", re.compile(r"igemm_|grouped_conv|naive_conv|MIOpen|miopen|SubTensorOp", re.I)),
    ("gemm", re.compile(r"Cijk_|gemm|Gemm|hipblaslt|_MT\d+x\d+", re.I)),
    ("attn_fwd", re.compile(r"attn_fwd(16)?_k")),
    ("decode_attn", re.compile(r"decode_attn_k|decode_combine_k")),
    ("kv_append", re.compile(r"kv_append_k")),
    ("attn_bwd_dkdv", re.compile(r"attn_bwd_dkdv(16)?_k")),
    ("attn_bwd_dq", re.compile(r"attn_bwd_dq(16)?_k")),
    ("attn_delta", re.compile(r"attn_delta_k")),
    ("rmsnorm", re.compile(r"rmsnorm|col_reduce")),
    ("swiglu", re.compile(r"swiglu")),
    ("rope", re.compile(r"rope")),
    ("xent", re.compile(r"xent|cross_entropy")),
    ("embedding", re.compile(r"embed")),
    ("optimizer", re.compile(r"adamw|sgd_k|sumsq")),
    ("rccl", re.compile(r"ncclDevKernel|rccl|nccl", re.I)),
    ("batchnorm(dph)", re.compile(r"bn_(stats|apply|finalize|merge|bwd)")),
    ("conv1x1(dph)", re.compile(r"ts_nt_k|ts_tn_k|ts_reduce|conv1x1")),
    ("conv3x3(dph)", re.compile(r"conv3_k|c3w_k|conv3x3|conv3_dgrad_w|conv_s2")),
    ("copy/fill", re.compile(r"copy|fill|FillFunctor|direct_copy", re.I)),
    ("elementwise(aten)", re.compile(r"elementwise|vectorized|reduce_kernel", re.I)),
]


def short_name(name: str) -> str:
    # demangled names carry "(anonymous namespace)" before the argument list: drop it, then cut the arguments
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n[:120]


def category(name: str) -> str:
    for cat, rx in CATEGORIES:
        if rx.search(name):
            return cat
    return "other"


def load_events(path: str):
    """-> list of (name, start_ns, end_ns)."""
    dbs = glob.glob(os.path.join(path, "**", "*_results.db"), recursive=True) if os.path.isdir(path) else [path]
    dbs = [d for d in dbs if d.endswith(".db")]
    if dbs:
        ev = []
        for db in dbs:
            con = sqlite3.connect(db)
            ev += list(con.execute("select name, start, end from kernels"))
            con.close()
        return ev
    csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    ev = []
    for f in csvs:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                ev.append((row["Kernel_Name"], int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    return ev


def marker_window(events, marker: str, run_steps: int, steps: int):
    """Events from the end of the marker launch that closes step (run_steps - steps) on, or None without markers.
    `events` sorted by start."""
    names = marker.split("|")
    idx = [i for i, e in enumerate(events) if any(n in e[0] for n in names)]
    if not idx or run_steps <= 0:
        return None
    per_step = max(1, round(len(idx) / run_steps))
    keep = steps * per_step
    if len(idx) <= keep:
        return events
    t0 = events[idx[-keep - 1]][2]   # end of the previous step's last marker launch
    return [e for e in events if e[1] >= t0]


def summarise(events, last_ms: float | None = None, steps: int = 1, top: int = 80, marker: str | None = None,
              run_steps: int = 0, step_ms: float | None = None):
    if not events:
        raise SystemExit("no kernel events found")
    events.sort(key=lambda e: e[1])
    win = marker_window(events, marker, run_steps, steps) if marker else None
    if win is not None:
        events = win
    elif last_ms:
        t_end = max(e[2] for e in events)
        events = [e for e in events if e[1] >= t_end - last_ms * 1e6]
    span = (max(e[2] for e in events) - min(e[1] for e in events)) / 1e6
    per_k = defaultdict(lambda: [0, 0.0])
    per_c = defaultdict(float)
    for name, s, e in events:
        d = (e - s) / 1e6
        k = short_name(name)
        per_k[k][0] += 1
        per_k[k][1] += d
        per_c[category(name)] += d
    busy = sum(per_c.values())
    launches = sum(c for c, _ in per_k.values())
    out = {
        "window": "marker" if win is not None else ("last_ms" if last_ms else "all"),
        "launches_per_step": round(launches / steps, 2),
        "idle_pct": round(100 * max(0.0, span - busy) / span, 2) if span > 0 else 0.0,
        "steps": steps,
        "span_ms_per_step": round(span / steps, 3),
        "kernel_busy_ms_per_step": round(busy / steps, 3),
        "categories_ms_per_step": {c: round(v / steps, 3) for c, v in sorted(per_c.items(), key=lambda x: -x[1])},
        "top_kernels": [
            {"name": k, "calls_per_step": round(c / steps, 2), "ms_per_step": round(t / steps, 3),
             "pct": round(100 * t / busy, 2)}
            for k, (c, t) in sorted(per_k.items(), key=lambda x: -x[1][1])[:top]
        ],
    }
    if step_ms:
        out["step_ms"] = step_ms
        out["idle_vs_step_pct"] = round(100 * max(0.0, step_ms - busy / steps) / step_ms, 2)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("path", help="rocprofv3 output directory, .db file, or CSV directory")
    ap.add_argument("--steps", type=int, default=1, help="divide totals by this many steps")
    ap.add_argument("--last-ms", type=float, default=None, help="only the last N ms of GPU activity")
    ap.add_argument("--json", default=None)
    ap.add_argument("--top", type=int, default=25, help="kernels printed (the JSON keeps up to 80)")
    ap.add_argument("--step-marker", default=None, help="kernel-name substring(s), '|'-separated, launched a fixed "
                    "number of times per step (e.g. adamw_k|sgd_k): count steps by it instead of a time window")
    ap.add_argument("--run-steps", type=int, default=0, help="steps the traced run executed (warm-up + timed)")
    ap.add_argument("--step-ms", type=float, default=None, help="un-traced ms/step: report idle vs the real step")
    args = ap.parse_args(argv)
    out = summarise(load_events(args.path), args.last_ms, args.steps, marker=args.step_marker,
                    run_steps=args.run_steps, step_ms=args.step_ms)
    extra = f", idle vs the un-traced {out['step_ms']} ms step {out['idle_vs_step_pct']} %" if "step_ms" in out else ""
    print(f"span/step {out['span_ms_per_step']} ms, kernel busy/step {out['kernel_busy_ms_per_step']} ms, "
          f"idle {out['idle_pct']} %, {out['launches_per_step']} launches/step ({out['window']} window){extra}")
    for c, v in out["categories_ms_per_step"].items():
        print(f"  {c:22s} {v:10.3f} ms")
    print("top kernels:")
    for k in out["top_kernels"][:args.top]:
        print(f"  {k['ms_per_step']:9.3f} ms {k['pct']:6.2f}% x{k['calls_per_step']:<7} {k['name'][:90]}")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
