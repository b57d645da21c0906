#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace stored as a rocpd SQLite database (`rocprofv3 --kernel-trace -d DIR -o NAME`
writes DIR/NAME_results.db on this ROCm): per-kernel time over the last --window fraction of the trace, the busy vs
span ratio (GPU idle = host-bound time) and the largest idle gaps.

    python benchmarks/rocpd_summary.py gpurun_out/prof_unet11/unet_results.db [--window 0.5] [--top 25]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=0.5, help="summarise the last fraction of the dispatches")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in c.execute("select id, coalesce(display_name, kernel_name) from rocpd_info_kernel_symbol")}
    rows = sorted(c.execute("select start, end, kernel_id from rocpd_kernel_dispatch"))
    rows = rows[int(len(rows) * (1 - a.window)):]
    if not rows:
        print("no dispatches")
        return
    span = (rows[-1][1] - rows[0][0]) / 1e6
    per = collections.defaultdict(lambda: [0.0, 0])
    busy, gaps, last_end = 0.0, [], rows[0][0]
    for s, e, k in rows:
        d = (e - s) / 1e6
        per[names.get(k, str(k))][0] += d
        per[names.get(k, str(k))][1] += 1
        if s > last_end:
            gaps.append(((s - last_end) / 1e6, names.get(k, str(k))[:60]))
        busy += max(0.0, (e - max(s, last_end)) / 1e6) if e > last_end else 0.0
        last_end = max(last_end, e)
    print(f"dispatches {len(rows)}, span {span:.3f} ms, kernel-busy {busy:.3f} ms ({100 * busy / span:.1f} %), "
          f"idle {span - busy:.3f} ms")
    print("top kernels (ms, share of busy, count):")
    for n, (t, cnt) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {t:9.3f}  {100 * t / busy:5.1f} %  x{cnt:<5d} {n[:110]}")
    print("largest idle gaps (ms, next kernel):")
    for g, n in sorted(gaps, reverse=True)[:10]:
        print(f"  {g:8.3f}  {n}")


if __name__ == "__main__":
    main()
