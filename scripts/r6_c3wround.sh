#!/bin/bash
# round 6: weight-gradient split count (workgroup slots per round the pixel-chunk splits fill, DPH_C3W_ROUND; the
# fp32 partials are s x N x K and re-read by ts_reduce_k) -- interleaved SimpleUNet and ResNet-50 benches
set -o pipefail
out=gpurun_out/r6c3w
mkdir -p $out
for r in 1 2; do
  for v in 512 256 384 1024; do
    DPH_C3W_ROUND=$v timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 60 --warmup 10 > $out/unet_${v}_r${r}.log 2>&1 || exit 1
    echo "unet $v r$r $(tail -1 $out/unet_${v}_r${r}.log | cut -c60-100)"
  done
  for v in 512 256 384 1024; do
    DPH_C3W_ROUND=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/resnet_${v}_r${r}.log 2>&1 || exit 1
    echo "resnet $v r$r $(tail -1 $out/resnet_${v}_r${r}.log | cut -c50-100)"
  done
done
