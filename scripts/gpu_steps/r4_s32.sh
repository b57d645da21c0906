#!/bin/bash
# round 4 step 32: ResNet-50 FSDP bf16 B=256 in-step A/B -- weight gradients on MIOpen / ts_tn_k (a) vs on c3w_k
# (1x1 identity rows, strided; 3x3 stays MIOpen: 0.82-0.91x per shape) (b), interleaved; SimpleUNet with the new c3w_k; profile of (b)
set -o pipefail
O=gpurun_out/r4s32; mkdir -p $O
A="DPH_W1_KERNEL=0 DPH_CONV3_WGRAD=miopen DPH_CONV_STRIDED_WGRAD=miopen"
B="DPH_W1_KERNEL=1 DPH_CONV3_WGRAD=miopen DPH_CONV_STRIDED_WGRAD=dph"
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_${v}_r$rep.log 2>&1 || { tail -20 $O/resnet_${v}_r$rep.log; exit 1; }
    echo "resnet $v rep=$rep $(grep '^{"metric' $O/resnet_${v}_r$rep.log | cut -c1-100)"
  done
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_r$rep.log 2>&1 || { tail -20 $O/unet_r$rep.log; exit 1; }
  echo "unet rep=$rep $(grep '^{"metric' $O/unet_r$rep.log | cut -c1-100)"
done
env $B bash scripts/prof_bench.sh $O/prof_resnet_b --layout resnet-fsdp 2>&1 | tail -30
