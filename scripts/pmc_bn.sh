#!/usr/bin/env bash
# HBM bytes of the BatchNorm / pooling / channel-sum kernels (benchmarks/bn_bench.py) from rocprofv3 PMC counters:
# one pass with FETCH_SIZE, one with WRITE_SIZE (the two do not fit one pass: 3 + 2 TCC counters > 4).
#   bash scripts/pmc_bn.sh OUTDIR
set -euo pipefail
out=${1:?usage: pmc_bn.sh OUTDIR}
mkdir -p "$out"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  raw=/tmp/pmc_bn_${ctr}_$$
  rm -rf "$raw"
  timeout -s KILL 120 rocprofv3 --pmc "$ctr" -d "$raw" -o p -- python benchmarks/bn_bench.py --batch 64 \
    > "$out/bn_bench_$ctr.log" 2>&1
  db=$(find "$raw" -name "*results.db" -print -quit)
  python benchmarks/pmc_summary.py "$db" --match "bn_|maxpool|chsum" --json "$out/pmc_$ctr.json" > "$out/pmc_$ctr.txt"
  head -n 30 "$out/pmc_$ctr.txt"
  rm -rf "$raw"
done
