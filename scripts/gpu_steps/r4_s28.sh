#!/bin/bash
# round 4 step 28: c3w_k with the LDS reads one k-step ahead of the MFMAs (scheduled), ring depth 2..5:
# 1x1 sweep (step 25's script) then 3x3 / strided / stem sweep (step 27's script)
set -o pipefail
sed -i 's#O=gpurun_out/r4s25#O=gpurun_out/r4s28/w1#; s#O = "gpurun_out/r4s25"#O = "gpurun_out/r4s28/w1"#' scripts/gpu_steps/r4_s25.sh
sed -i 's#O=gpurun_out/r4s27#O=gpurun_out/r4s28/c3#; s#O = "gpurun_out/r4s27"#O = "gpurun_out/r4s28/c3"#' scripts/gpu_steps/r4_s27.sh
bash scripts/gpu_steps/r4_s25.sh && bash scripts/gpu_steps/r4_s27.sh
