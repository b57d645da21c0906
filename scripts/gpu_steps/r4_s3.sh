#!/bin/bash
# round 4 step 3: staggered wgrad kernel (numerics, A/B), in-step A/Bs (wgrad 32 vs 33, NT fused vs all), UNet profiles
set -o pipefail
O=gpurun_out/r4s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn" \
  > $O/tests_wgrad.log 2>&1 || { tail -30 $O/tests_wgrad.log; exit 1; }
tail -2 $O/tests_wgrad.log
timeout -k 10 300 python -u benchmarks/gemm_mfma_ab.py --variants 32,33 --rounds 3 --json $O/wgrad_ab.json > $O/wgrad_ab.log 2>&1 || { tail $O/wgrad_ab.log; exit 1; }
grep -v amdgpu $O/wgrad_ab.log | grep -v "^{" | tail -8
for v in 33 32; do
  DPH_WGRAD_MFMA=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_wgrad$v.log 2>&1 || { tail -20 $O/bench_wgrad$v.log; exit 1; }
  tail -1 $O/bench_wgrad$v.log | cut -c1-200
done
DPH_WGRAD_MFMA=33 DPH_GEMM_NT=all timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_ntall.log 2>&1 || { tail -20 $O/bench_ntall.log; exit 1; }
tail -1 $O/bench_ntall.log | cut -c1-200
for prec in bf16 bf16-autocast; do
  bash scripts/prof_cmd.sh $O/unet_$prec 20 120 python bench.py --layout unet-ddp --unet-precision $prec --steps 20 --warmup 5 > $O/unet_prof_$prec.txt 2>&1 || { tail -20 $O/unet_prof_$prec.txt; exit 1; }
  head -25 $O/unet_prof_$prec.txt
done
