set -o pipefail
mkdir -p gpurun_out/r5/gemm_power
timeout -k 10 400 python3 -u benchmarks/probes/gemm_power.py --json gpurun_out/r5/gemm_power/gemm_power.json > gpurun_out/r5/gemm_power/gemm_power.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 3 --quiet > gpurun_out/r5/gemm_power/bench_fused_r$r.log 2>&1 || exit 1
  DPH_GEMM_NT=all timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 3 --quiet > gpurun_out/r5/gemm_power/bench_ntall_r$r.log 2>&1 || exit 1
done
