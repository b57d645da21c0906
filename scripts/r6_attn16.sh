#!/bin/bash
# round-6: 16x16x32 attention kernels -- numerics vs fp32, then interleaved A/B (variant 0 = 16x16x32, 1 = 32x32x16)
# and per-kernel times under rocprofv3
set -o pipefail
out=gpurun_out/r6_attn16
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or rope_attention" tests/test_attention_dropout.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 120 python -u benchmarks/probes/attn_one.py --iters 20 --variant $v > $out/ab_v${v}_r$r.log 2>&1 || exit 1
    echo "v$v r$r: $(tr '\n' ' ' < $out/ab_v${v}_r$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_v$v -o p -- python3 $GRAFT_REPO_ROOT/benchmarks/probes/attn_one.py --iters 10 --variant $v > $GRAFT_REPO_ROOT/$out/prof_v$v.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for v in 0 1; do f=$(find $out/prof_v$v -name "*kernel_stats.csv" | head -1); echo "== v$v"; cut -d, -f1-4 "$f" | grep -i attn; done
