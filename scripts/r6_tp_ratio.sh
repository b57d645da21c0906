#!/bin/bash
# round 6, final tree: the 1-GPU 7B step and one TP rank at TP 8 / 4 on the same box (ratio to the ideal 1/tp share)
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6tpr
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > $out/bench.log 2>&1 || exit 1
ms1=$(python3 -c "import json; print([json.loads(l) for l in open('$out/bench.log') if l.startswith('{')][-1]['ms_per_step'])")
echo "1-GPU step: $ms1 ms"
for tp in 8 4; do
  timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp $tp --steps 5 > $out/tp${tp}.log 2>&1 || exit 1
  ms=$(python3 -c "import json; print([json.loads(l) for l in open('$out/tp${tp}.log') if l.startswith('{')][-1]['ms_per_step'])")
  python3 -c "print('tp $tp: $ms ms/step, ideal', round($ms1 / $tp, 1), 'ratio', round($ms * $tp / $ms1, 3))"
done
