#!/bin/bash
# round 6: SimpleUNet up-path weight / bias gradients written straight into the engine's buckets -- tests, bench x3
set -o pipefail
out=gpurun_out/r6unet2
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_upsample_gpu.py \
  tests/test_whole_net_grad_gpu.py tests/test_bn_epilogue_gpu.py -k "unet or up_concat or upsample" > $out/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 60 --warmup 10 > $out/unet_r${r}.log 2>&1 || exit 1
  echo "r$r $(tail -1 $out/unet_r${r}.log | cut -c60-140)"
done
