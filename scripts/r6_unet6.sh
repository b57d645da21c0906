#!/bin/bash
# round 6: SimpleUNet encoder blocks: skip gradient added in the max pooling gather + its last BatchNorm reduction there
# -- tests, then interleaved unet-ddp A/B of just those three folds (DPH_UNET_SKIP_FOLD)
set -o pipefail
out=gpurun_out/r6unet6
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_whole_net_grad_gpu.py > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  for v in 0 1; do
    DPH_UNET_SKIP_FOLD=$v timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 60 --warmup 10 > $out/unet_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/unet_v${v}_r${r}.log | cut -c60-140)"
  done
done
