#!/bin/bash
# round 4 step 1: numerics of the 32x32x16 NT kernel (+ ragged shapes), then the shape A/B against hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py \
  > gpurun_out/r4_s1_tests.log 2>&1 || { tail -30 gpurun_out/r4_s1_tests.log; exit 1; }
tail -3 gpurun_out/r4_s1_tests.log
timeout -k 10 400 python -u benchmarks/gemm_nt_bench.py --variants 1,3 --rounds 3 --json gpurun_out/r4_s1_ntbench.json \
  > gpurun_out/r4_s1_ntbench.log 2>&1
rc=$?
cat gpurun_out/r4_s1_ntbench.log | grep -v amdgpu.ids
exit $rc
