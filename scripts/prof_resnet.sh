#!/usr/bin/env bash
# ResNet-50 FSDP bf16 step (examples/resnet_benchmark.py) under rocprofv3 --kernel-trace: per-kernel / per-category
# summary of the last STEPS steps.  Raw rocprof output stays in /tmp; the summary lands in OUTDIR.
#
#   bash scripts/prof_resnet.sh gpurun_out/prof_resnet [batch] [steps]
set -euo pipefail
out=${1:?usage: prof_resnet.sh OUTDIR [batch] [steps]}
B=${2:-256}
S=${3:-10}
mkdir -p "$out"
export TMPDIR=/tmp
raw=/tmp/prof_resnet_$$
rm -rf "$raw"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$raw" -o p -- python examples/resnet_benchmark.py --device cuda \
  --arch resnet50 --use-fsdp --amp --channels-last --batch-size "$B" --epochs 2 --steps-syn "$S" \
  > "$out/resnet_under_rocprof.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
# the last epoch: S steps at ~MS_PER_IMG ms per image (default 0.0905 = 11.05k img/s; trimmed so no part of the
# previous epoch is counted)
ms=$(python -c "print(0.97 * $S * $B * ${MS_PER_IMG:-0.0905})")
python benchmarks/prof_summary.py "$db" --steps "$S" --last-ms "$ms" --step-marker "sgd_k" --run-steps $((2 * S)) \
  --json "$out/summary.json" > "$out/summary.txt"
head -n 40 "$out/summary.txt"
rm -rf "$raw"
