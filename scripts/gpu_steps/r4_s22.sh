#!/bin/bash
# round 4 step 22: the 7B step with the dK/dV priority variant (default 6) vs the previous default 2, interleaved;
# then a profile of the default step
set -o pipefail
O=gpurun_out/r4s22; mkdir -p $O
for rep in 1 2; do
  for v in 2 6; do
    DPH_ATTN_BWD_VAR=$v timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 2>&1 | tee $O/bench_bwdvar${v}_r$rep.log | grep --line-buffered "^{" | cut -c1-120
  done
done
bash scripts/prof_bench.sh $O/prof_7b 2>&1 | tail -30
