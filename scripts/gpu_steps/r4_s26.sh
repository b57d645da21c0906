#!/bin/bash
# round 4 step 26 = steps 25 + 24 in one call (no box was free for 24)
set -o pipefail
bash scripts/gpu_steps/r4_s25.sh && bash scripts/gpu_steps/r4_s24.sh
