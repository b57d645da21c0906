#!/bin/bash
# round 6: projection shortcut's two BatchNorm dx passes fused -- tests, interleaved ResNet-50 A/B (DPH_BN_DUAL_DX)
set -o pipefail
out=gpurun_out/r6dx
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_whole_net_grad_gpu.py > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in 0 1; do
    DPH_BN_DUAL_DX=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 40 --warmup 5 > $out/bench_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/bench_v${v}_r${r}.log | cut -c60-140)"
  done
done
