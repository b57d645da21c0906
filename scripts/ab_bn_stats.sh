#!/usr/bin/env bash
# A/B of the BN statistics / backward-reduce kernels' block combine (DPH_BN_TREE=0 serial vs 1 LDS tree) under rocprofv3 --kernel-trace
# over benchmarks/bn_bench.py, plus the GPU BN tests with the tree merge.
#   bash scripts/ab_bn_stats.sh OUTDIR
set -euo pipefail
out=${1:?usage: ab_bn_stats.sh OUTDIR}
mkdir -p "$out"
export TMPDIR=/tmp
for t in 0 1; do
  raw=/tmp/ab_bn_${t}_$$
  rm -rf "$raw"
  DPH_BN_TREE=$t timeout -k 10 200 rocprofv3 --kernel-trace -d "$raw" -o p -- python benchmarks/bn_bench.py \
    > "$out/bn_bench_tree$t.log" 2>&1
  db=$(find "$raw" -name "*results.db" -print -quit)
  python benchmarks/prof_summary.py "$db" --json "$out/summary_tree$t.json" > "$out/summary_tree$t.txt"
  grep -E "bn_stats|finalize" "$out/summary_tree$t.txt" | head -8
  rm -rf "$raw"
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs.py -x -q -k "bn or resnet or bottleneck or unet or conv" \
  --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
tail -n 1 "$out/tests.log"
