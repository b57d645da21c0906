#!/bin/bash
# round 6, final tree: one TP rank's step (collectives stubbed) at TP 8 and 4 -- timing twice, then a kernel profile
# whose step window is counted by the AdamW launches
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6tp
mkdir -p $out
for tp in 8 4; do
  for r in 1 2; do
    timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp $tp --steps 5 > $out/tp${tp}_bench_r$r.log 2>&1 || exit 1
    echo "tp $tp r$r: $(tail -1 $out/tp${tp}_bench_r$r.log | cut -c1-200)"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_tp$tp -o p -- python3 $R/benchmarks/tp_rank_bench.py --tp $tp --steps 3 --warmup 2 > $out/tp${tp}_prof.log 2>&1 || exit 1
  db=$(find /tmp/prof_tp$tp -name "*results.db" -print -quit)
  python3 $R/benchmarks/prof_summary.py "$db" --steps 3 --step-marker "adamw_k" --run-steps 5 --json $out/summary_tp$tp.json > $out/summary_tp$tp.txt || exit 1
  rm -rf /tmp/prof_tp$tp
  head -16 $out/summary_tp$tp.txt | cut -c1-150
done
