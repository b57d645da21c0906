#!/usr/bin/env bash
# Interleaved same-box A/B of bench.py between this tree and another checkout (with its own built _C.so).
#   bash scripts/ab_bench.sh OTHER_TREE OUTDIR [rounds] [extra bench args...]
set -euo pipefail
other=${1:?other tree}
out=${2:?outdir}
rounds=${3:-2}
shift 3 || true
mkdir -p "$out"
for i in $(seq 1 "$rounds"); do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 "$@" > "$out/new_$i.log" 2>&1
  grep '^{"metric"' "$out/new_$i.log"
  (cd "$other" && timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 "$@") > "$out/old_$i.log" 2>&1
  grep '^{"metric"' "$out/old_$i.log"
done
