#!/usr/bin/env bash
# round 3 step 32: weight-gradient GEMM epilogue through LDS (16-B row stores) vs per-element stores
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s32_tests_lds 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn or wgrad or ragged" || exit 1
DPH_WGRAD_EPI=scalar run r3_s32_tests_scalar 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn or wgrad or ragged" || exit 1
for rep in 1 2; do
  DPH_WGRAD_EPI=scalar run r3_s32_bench_scalar_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  run r3_s32_bench_lds_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
done
