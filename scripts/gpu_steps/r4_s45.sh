#!/bin/bash
# round 4 step 45: default 7B bench twice on one box (box-to-box spread check after step 44's 27 537) + kernel profile
set -o pipefail
O=gpurun_out/r4s45; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_r$rep.log 2>&1 || { tail -20 $O/bench_r$rep.log; exit 1; }
  echo "7b rep=$rep $(grep -o '"value": [0-9.]*' $O/bench_r$rep.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_r$rep.log)"
done
bash scripts/prof_bench.sh $O/prof_7b 2>&1 | tail -22
