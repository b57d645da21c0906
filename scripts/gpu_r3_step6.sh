#!/usr/bin/env bash
# round 3 step 6: the whole GPU tier + ring-merge microbench
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/r3_s6_gpu_tier.log 2>&1; rc=$?; echo "gpu tier rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u benchmarks/ring_merge_bench.py --json gpurun_out/r3_ring_merge_bench.json > gpurun_out/r3_ring_merge_bench.log 2>&1; echo "ring bench rc=$?"
