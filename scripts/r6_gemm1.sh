#!/bin/bash
# round 6: deep-K 1x1 convolutions on the LDS-DMA one-tap GEMM -- tests, interleaved ResNet-50 A/B (DPH_GEMM1_LDS=0 vs
# default), kernel profile
set -o pipefail
out=gpurun_out/r6g1
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_whole_net_grad_gpu.py tests/test_strided_conv_gpu.py tests/test_kernels_gpu.py \
  -k "bn or conv or bottleneck or slot or resnet or epilogue or mask or dual or whole or pool or deep or ts_gemm" > $out/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in 0 1; do
    DPH_GEMM1_LDS=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/bench_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/bench_v${v}_r${r}.log | cut -c60-140)"
  done
done
timeout -k 10 500 bash scripts/prof_resnet.sh $out/prof 256 10 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -10 $out/prof/summary.txt | cut -c1-150
