#!/bin/bash
# round 4 step 23: SimpleUNet profile after the launch cuts (conv-epilogue statistics, bf16 bias, bucket bias grads)
set -o pipefail
O=gpurun_out/r4s23; mkdir -p $O
bash scripts/prof_bench.sh $O/prof_unet --layout unet-ddp 2>&1 | tail -45
