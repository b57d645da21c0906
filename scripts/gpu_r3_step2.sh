timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py > gpurun_out/r3_gemm_nt_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 400 python -u benchmarks/gemm_nt_bench.py --json gpurun_out/r3_gemm_nt_bench.json > gpurun_out/r3_gemm_nt_bench.log 2>&1; rc2=$?; echo "bench rc=$rc2"
  if [ $rc -eq 0 ] && [ $rc2 -eq 0 ]; then
    DPH_FUSED_MLP=1 DPH_FUSED_QKV=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_fused_v1.log 2>&1; echo "bench.py rc=$?"
  fi
fi
