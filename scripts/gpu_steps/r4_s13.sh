#!/bin/bash
# round 4 step 13: GPU tests of this round's kernels (dQ variant, UNet conv-epilogue statistics, 1x1 LDS-DMA weight
# gradient, strided convs, RGB stem) and their microbenchmarks
set -o pipefail
O=gpurun_out/r4s13; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_strided_conv_gpu.py tests/test_kernels_gpu.py tests/test_upsample_gpu.py \
  -k "Strided or strided or stem or sub or dq_variants or flash_attention or unet or bias_conv or Unet or conv1x1 or ts_gemm_tn or bottleneck" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1; do
  DPH_W1_KERNEL=$v timeout -k 10 200 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_$v.json $([ $v = 1 ] && echo --miopen) > $O/w1_$v.log 2>&1 || { tail -20 $O/w1_$v.log; exit 1; }
  grep -v amdgpu $O/w1_$v.log
done
timeout -k 10 200 python -u benchmarks/stem_conv_bench.py > $O/stem.log 2>&1 || { tail -20 $O/stem.log; exit 1; }
grep -v amdgpu $O/stem.log | tail -8
for rep in 1 2 3; do
  for v in 0 2; do
    DPH_ATTN_DQ_VAR=$v timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which bwd --iters 20 > $O/bwd_dq${v}_r$rep.log 2>&1 || { tail $O/bwd_dq${v}_r$rep.log; exit 1; }
    echo "dq=$v rep=$rep $(grep -v amdgpu $O/bwd_dq${v}_r$rep.log | tail -1)"
  done
done
