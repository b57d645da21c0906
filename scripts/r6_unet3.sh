#!/bin/bash
# round 6: SimpleUNet up-path direct gradient writes, interleaved A/B (DPH_UPCAT_DIRECT=0 vs 1)
set -o pipefail
out=gpurun_out/r6unet3
mkdir -p $out
for r in 1 2 3; do
  for v in 0 1; do
    DPH_UPCAT_DIRECT=$v timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 60 --warmup 10 > $out/unet_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/unet_v${v}_r${r}.log | cut -c60-140)"
  done
done
