#!/bin/bash
# round 4 step 10: strided convolutions on the gathered implicit-GEMM kernels -- numerics, ResNet-50 A/B vs MIOpen,
# ResNet-50 profile
set -o pipefail
O=gpurun_out/r4s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_strided_conv_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for st in 0 1; do
    DPH_CONV_STRIDED=$st timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_strided${st}_r$rep.log 2>&1 || { tail -20 $O/resnet_strided${st}_r$rep.log; exit 1; }
    echo "strided=$st rep=$rep $(tail -1 $O/resnet_strided${st}_r$rep.log | cut -c1-110)"
  done
done
bash scripts/prof_bench.sh $O/prof_resnet --layout resnet-fsdp
