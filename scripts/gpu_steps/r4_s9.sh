#!/bin/bash
# round 4 step 9: new async-TP / conv-routing GPU tests, fresh 7B step profile on the round-4 tree
set -o pipefail
O=gpurun_out/r4s9; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_async_tp_gpu.py \
  tests/test_kernels_gpu.py tests/test_upsample_gpu.py -k "async or conv or unet or Conv or Unet or bias" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/prof_bench.sh $O/prof_7b
