#!/bin/bash
# round 4 step 12: strided convs with the sub-image dgrad hand-off + MIOpen wgrad -- tests, ResNet-50 A/B, profile;
# SimpleUNet eager vs whole-step HIP graph
set -o pipefail
O=gpurun_out/r4s12; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_strided_conv_gpu.py \
  tests/test_kernels_gpu.py -k "strided or Strided or bottleneck or sub or conv1x1" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for st in 0 1; do
    DPH_CONV_STRIDED=$st timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_strided${st}_r$rep.log 2>&1 || { tail -20 $O/resnet_strided${st}_r$rep.log; exit 1; }
    echo "strided=$st rep=$rep $(tail -1 $O/resnet_strided${st}_r$rep.log | cut -c1-110)"
  done
done
bash scripts/prof_bench.sh $O/prof_resnet --layout resnet-fsdp
for g in 0 1; do
  flag=""; [ $g = 1 ] && flag=--graph
  timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 $flag > $O/unet_graph$g.log 2>&1 || { tail -20 $O/unet_graph$g.log; exit 1; }
  echo "unet graph=$g $(tail -1 $O/unet_graph$g.log | cut -c1-110)"
done
