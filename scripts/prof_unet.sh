#!/usr/bin/env bash
# SimpleUNet DDP step (bench.py --layout unet-ddp, B=4, 65 x 181 x 360, bf16) un-traced, then under
# rocprofv3 --kernel-trace: per-kernel / per-category summary of the last STEPS steps, counted by the fused AdamW
# launches (one per step), with the un-traced step time for the host-gap share.  Raw rocprof output stays in /tmp.
#
#   bash scripts/prof_unet.sh OUTDIR [steps] [warmup]
set -euo pipefail
out=${1:?usage: prof_unet.sh OUTDIR [steps] [warmup]}
S=${2:-20}
W=${3:-10}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --layout unet-ddp --steps 50 --warmup "$W" > "$out/bench.log" 2>&1
step_ms=$(python -c "import json; print([json.loads(l) for l in open('$out/bench.log') if l.startswith('{')][-1]['ms_per_step'])")
raw=/tmp/prof_unet_$$
rm -rf "$raw"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$raw" -o p -- python bench.py --layout unet-ddp --steps "$S" \
  --warmup "$W" --no-telemetry > "$out/bench_under_rocprof.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
python benchmarks/prof_summary.py "$db" --steps "$S" --step-marker adamw --run-steps $((S + W)) \
  --step-ms "$step_ms" --json "$out/summary.json" > "$out/summary.txt"
head -n 45 "$out/summary.txt"
rm -rf "$raw"
