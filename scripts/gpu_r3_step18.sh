#!/usr/bin/env bash
# round 3 step 18: 3x3 kernel with 4- vs 8-wave tiles (parity + per-pass bench)
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for wm in 2 4; do
  DPH_CONV3_WM=$wm run r3_s18_tests_wm$wm python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_upsample_gpu.py -k "conv3x3 or bottleneck or unet" || exit 1
done
for wm in 2 4; do
  DPH_CONV3_WM=$wm run r3_s18_bench_wm$wm python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench_wm$wm.json || exit 1
done
