#!/bin/bash
# round 4 step 14: SimpleUNet BN statistics from the 3x3 conv epilogue -- tests, A/B, profile
set -o pipefail
O=gpurun_out/r4s14; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_upsample_gpu.py \
  -k "unet or bias_conv or Unet" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for st in 0 1; do
    DPH_UNET_CONV_STATS=$st timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_stats${st}_r$rep.log 2>&1 || { tail -20 $O/unet_stats${st}_r$rep.log; exit 1; }
    echo "stats=$st rep=$rep $(tail -1 $O/unet_stats${st}_r$rep.log | cut -c1-110)"
  done
done
bash scripts/prof_bench.sh $O/prof_unet --layout unet-ddp
