#!/bin/bash
# round 4 step 21: issue priority over the MFMA chains in the dQ and forward kernels -- numerics, A/B
set -o pipefail
O=gpurun_out/r4s21; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "priority_variants" \
  2>&1 | tee $O/tests.log | tail -2
for rep in 1 2 3; do
  for cfg in "6 2 0" "6 3 1"; do
    set -- $cfg
    DPH_ATTN_BWD_VAR=$1 DPH_ATTN_DQ_VAR=$2 DPH_ATTN_FWD_PRIO=$3 timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which fwd,bwd --iters 20 2>&1 \
      | tee $O/attn_${1}_${2}_${3}_r$rep.log | grep --line-buffered "fwd\|bwd" | tr '\n' ' ' | sed "s/^/bwdvar=$1 dq=$2 fwdprio=$3 rep=$rep /"; echo
  done
done
