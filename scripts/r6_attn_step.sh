#!/bin/bash
# round-6: attention variants in the 7B step's layout (packed QKV views) and under the step profile
set -o pipefail
out=gpurun_out/r6_attn_step
mkdir -p $out
for r in 1 2; do
  for v in 0 2; do
    timeout -k 10 120 python -u benchmarks/probes/attn_one.py --iters 20 --variant $v --packed > $out/ab_packed_v${v}_r$r.log 2>&1 || exit 1
    echo "packed v$v r$r: $(grep -v amdgpu.ids $out/ab_packed_v${v}_r$r.log | tr '\n' ' ')"
  done
done
bash scripts/prof_bench.sh $out/prof_v0 > /dev/null || exit 1
bash scripts/prof_bench.sh $out/prof_v2 --attn-variant 2 > /dev/null || exit 1
for v in 0 2; do echo "== step v$v"; head -3 $out/prof_v$v/summary.txt; grep -E "attn" $out/prof_v$v/summary.txt | head -8; done
