#!/bin/bash
# round 4 step 20: dK/dV kernel with issue priority over its MFMA chains (DPH_ATTN_BWD_VAR=6) -- numerics, A/B vs 2
set -o pipefail
O=gpurun_out/r4s20; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "priority_variant" \
  2>&1 | tee $O/tests.log | tail -2
for rep in 1 2 3; do
  for v in 2 6; do
    DPH_ATTN_BWD_VAR=$v timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which bwd --iters 20 2>&1 | tee $O/bwd_v${v}_r$rep.log | grep --line-buffered "bwd" | sed "s/^/v=$v rep=$rep /"
  done
done
