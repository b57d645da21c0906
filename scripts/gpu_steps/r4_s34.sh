#!/bin/bash
# round 4 step 34: weight gradients on c3w_k by default (1x1 identity rows, 3x3, strided; one resident round of split-K)
# -- conv / model GPU tests, ResNet-50 in-step A/B vs the old MIOpen / ts_tn_k defaults, SimpleUNet, profile
set -o pipefail
O=gpurun_out/r4s34; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_strided_conv_gpu.py tests/test_graphs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="DPH_W1_KERNEL=0 DPH_CONV3_WGRAD=miopen DPH_CONV_STRIDED_WGRAD=miopen"
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then E=$A; else E="DPH_NOTHING=1"; fi
    env $E timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_${v}_r$rep.log 2>&1 || { tail -20 $O/resnet_${v}_r$rep.log; exit 1; }
    echo "resnet $v rep=$rep $(grep '^{"metric' $O/resnet_${v}_r$rep.log | cut -c1-100)"
  done
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_r$rep.log 2>&1 || { tail -20 $O/unet_r$rep.log; exit 1; }
  echo "unet rep=$rep $(grep '^{"metric' $O/unet_r$rep.log | cut -c1-100)"
done
bash scripts/prof_bench.sh $O/prof_resnet --layout resnet-fsdp 2>&1 | tail -30
