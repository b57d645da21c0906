#!/usr/bin/env python3
"""Per-kernel PMC counter summary from rocprofv3's rocpd SQLite output (``rocprofv3 --pmc ... -d DIR -o p``).

Prints, for every kernel whose name matches ``--match``, the mean per dispatch of each collected counter plus the
derived ratios the CDNA4 guide uses (MFMA busy share of cycles, wait shares, LDS conflict rate, effective clock).

    python benchmarks/pmc_summary.py gpurun_out/x/pmc1/p_results.db [--match attn] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import re
import sqlite3
from collections import defaultdict


def load(db: str, match: str):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration, vgpr_count, accum_vgpr_count, "
                     "sgpr_count, lds_block_size from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value (summed over dims)
    meta = {}
    for disp, name, ctr, val, dur, vg, ag, sg, lds in rows:
        if match and not re.search(match, name):
            continue
        short = re.sub(r"\(.*", "", name)[:90]
        per[(short, disp)][ctr] += float(val)
        meta[short] = dict(vgpr=vg, agpr=ag, sgpr=sg, lds=lds)
        per[(short, disp)]["_dur_ns"] = float(dur)
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _), d in per.items():
        for ctr, v in d.items():
            agg[k][ctr].append(v)
    out = {}
    for k, d in agg.items():
        m = {ctr: sum(v) / len(v) for ctr, v in d.items()}
        m["_dispatches"] = len(d["_dur_ns"])
        m.update(meta[k])
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if key in m:
                    m[key + "/WAVE_CYCLES"] = m[key] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
            # MFMA busy cycles are summed over SIMDs; busy cycles per SE -> normalise by SIMDs per SE (256 CUs*4/32)
            m["mfma_busy_per_simd_share"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] * 32)
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_share"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "GRBM_GUI_ACTIVE" in m and m["_dur_ns"] > 0:
            m["eff_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / m["_dur_ns"]
        out[k] = m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    merged: dict = defaultdict(dict)
    for db in a.dbs:
        for k, m in load(db, a.match).items():
            merged[k].update(m)
    for k, m in sorted(merged.items()):
        print(f"== {k}")
        for ctr in sorted(m):
            v = m[ctr]
            print(f"   {ctr:40s} {v:.6g}" if isinstance(v, float) else f"   {ctr:40s} {v}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(merged, fh, indent=1)


if __name__ == "__main__":
    main()
