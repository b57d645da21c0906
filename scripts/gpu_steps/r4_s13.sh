#!/bin/bash
# round 4 step 13: dQ kernel without register spills (quarter-sub-tile K / V read-ahead) -- numerics, A/B
set -o pipefail
O=gpurun_out/r4s13; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dq_variants or flash_attention" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in 0 2; do
    DPH_ATTN_DQ_VAR=$v timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which bwd --iters 20 > $O/bwd_dq${v}_r$rep.log 2>&1 || { tail $O/bwd_dq${v}_r$rep.log; exit 1; }
    echo "dq=$v rep=$rep $(grep -v amdgpu $O/bwd_dq${v}_r$rep.log | tail -1)"
  done
done
