#!/bin/bash
# round 6 (second pass): the ResNet-50 test, then the remaining BN / conv tests, interleaved A/B, profile
set -o pipefail
out=gpurun_out/r6bn
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_strided_conv_gpu.py tests/test_whole_net_grad_gpu.py \
  "tests/test_kernels_gpu.py" -k "bn or bottleneck or resnet or conv or epilogue or slot" > $out/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for v in 0 1; do
    DPH_BN_EPILOGUE=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/bench_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/bench_v${v}_r${r}.log | cut -c1-200)"
  done
done
timeout -k 10 500 bash scripts/prof_resnet.sh $out/prof 256 10 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -12 $out/prof/summary.txt
