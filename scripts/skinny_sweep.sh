#!/usr/bin/env bash
# Skinny-GEMM configuration sweep (waves per workgroup x unroll) on the 7B decode projections.
#   bash scripts/skinny_sweep.sh OUTDIR
set -euo pipefail
out=${1:?outdir}
mkdir -p "$out"
for cfg in default 8,8 8,4 4,8 4,4 2,8 2,4; do
  if [ "$cfg" = default ]; then unset DPH_SKINNY_CFG; else export DPH_SKINNY_CFG=$cfg; fi
  timeout -k 10 120 python -u benchmarks/skinny_gemm_bench.py --ms 4 8 16 --json "$out/skinny_${cfg/,/_}.json" \
    > "$out/skinny_${cfg/,/_}.log" 2>&1
done
