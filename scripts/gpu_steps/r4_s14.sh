#!/bin/bash
# round 4 step 14: in-step A/B of the chunk-tap stem and the UNet BN
# statistics from the conv epilogue) and a ResNet-50 profile of the result
set -o pipefail
O=gpurun_out/r4s14; mkdir -p $O
for rep in 1 2; do
  for cfg in "0 1" "0 0"; do
    set -- $cfg
    tag=w1$1_stem$2
    DPH_W1_KERNEL=$1 DPH_STEM_KERNEL=$2 timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_${tag}_r$rep.log 2>&1 || { tail -20 $O/resnet_${tag}_r$rep.log; exit 1; }
    echo "resnet $tag rep=$rep $(tail -1 $O/resnet_${tag}_r$rep.log | cut -c1-110)"
  done
done
for rep in 1 2; do
  for st in 0 1; do
    DPH_UNET_CONV_STATS=$st timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_stats${st}_r$rep.log 2>&1 || { tail -20 $O/unet_stats${st}_r$rep.log; exit 1; }
    echo "unet stats=$st rep=$rep $(tail -1 $O/unet_stats${st}_r$rep.log | cut -c1-110)"
  done
done
bash scripts/prof_bench.sh $O/prof_resnet --layout resnet-fsdp
