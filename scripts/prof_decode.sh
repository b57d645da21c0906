#!/usr/bin/env bash
# Per-kernel profile of eager Llama decode steps (benchmarks/decode_bench.py) under rocprofv3 --kernel-trace.
#
#   bash scripts/prof_decode.sh OUTDIR BATCH [PROMPT] [MODE]      (MODE: eager (default) or graph)
set -euo pipefail
out=${1:?usage: prof_decode.sh OUTDIR BATCH [PROMPT]}
B=${2:?batch}
P=${3:-1024}
M=${4:-eager}
mkdir -p "$out"
export TMPDIR=/tmp
raw=/tmp/prof_decode_$$
rm -rf "$raw"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$raw" -o p -- python benchmarks/decode_bench.py --batches "$B" \
  --prompt "$P" --steps 32 --modes "$M" --json "$out/bench_b$B.json" > "$out/run_b$B.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
ms=$(python -c "import json,sys; print(32 * 0.98 * json.load(open(sys.argv[1]))['rows'][0][sys.argv[2] + '_ms_per_step'])" "$out/bench_b$B.json" "$M")
python benchmarks/prof_summary.py "$db" --steps 32 --last-ms "$ms" --json "$out/summary_b$B.json" > "$out/summary_b$B.txt"
head -n 30 "$out/summary_b$B.txt"
rm -rf "$raw"
