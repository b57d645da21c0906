#!/bin/bash
# round 4 step 29: step 28 (c3w_k read lookahead + ring depth sweeps) + SimpleUNet eager profile with marker-counted
# steps (prof_summary --step-marker)
set -o pipefail
bash scripts/gpu_steps/r4_s28.sh && bash scripts/prof_bench.sh gpurun_out/r4s29/prof_unet --layout unet-ddp 2>&1 | tail -25
