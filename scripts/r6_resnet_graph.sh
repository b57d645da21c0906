#!/bin/bash
# round 6: ResNet-50 FSDP bf16 B=256 -- eager vs whole-step HIP graph, interleaved
set -o pipefail
out=gpurun_out/r6rg
mkdir -p $out
for r in 1 2; do
  for g in no-graph graph; do
    timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 --$g > $out/${g}_r${r}.log 2>&1 || { tail -20 $out/${g}_r${r}.log; exit 1; }
    echo "$g r$r $(tail -1 $out/${g}_r${r}.log | cut -c60-150)"
  done
done
