#!/bin/bash
# round 6: cancelled conv-bias gradients zeroed once in persistent buckets -- tests, UNet kernel profile, bench x2
set -o pipefail
out=gpurun_out/r6unet4
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_whole_net_grad_gpu.py tests/test_dist_engine_gpu.py -k "unet or bias or engine or ddp" > $out/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 500 bash scripts/prof_unet.sh $out/prof 20 10 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -24 $out/prof/summary.txt | cut -c1-150
