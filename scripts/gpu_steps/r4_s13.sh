#!/bin/bash
# round 4 step 13: dQ kernel without register spills (A/B); SimpleUNet BN statistics from the conv epilogue (tests, A/B,
# profile); 1x1 weight gradient on the LDS-DMA kernel vs ts_tn_k vs MIOpen
set -o pipefail
O=gpurun_out/r4s13; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_upsample_gpu.py \
  -k "dq_variants or flash_attention or unet or bias_conv or Unet or conv1x1 or ts_gemm_tn or bottleneck" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1; do
  DPH_W1_KERNEL=$v timeout -k 10 200 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_$v.json $([ $v = 1 ] && echo --miopen) > $O/w1_$v.log 2>&1 || { tail -20 $O/w1_$v.log; exit 1; }
  grep -v amdgpu $O/w1_$v.log
done
for rep in 1 2 3; do
  for v in 0 2; do
    DPH_ATTN_DQ_VAR=$v timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which bwd --iters 20 > $O/bwd_dq${v}_r$rep.log 2>&1 || { tail $O/bwd_dq${v}_r$rep.log; exit 1; }
    echo "dq=$v rep=$rep $(grep -v amdgpu $O/bwd_dq${v}_r$rep.log | tail -1)"
  done
done
for rep in 1 2; do
  for st in 0 1; do
    DPH_UNET_CONV_STATS=$st timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_stats${st}_r$rep.log 2>&1 || { tail -20 $O/unet_stats${st}_r$rep.log; exit 1; }
    echo "unet stats=$st rep=$rep $(tail -1 $O/unet_stats${st}_r$rep.log | cut -c1-110)"
  done
done
for rep in 1 2; do
  for w in 0 1; do
    DPH_W1_KERNEL=$w timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_w1${w}_r$rep.log 2>&1 || { tail -20 $O/resnet_w1${w}_r$rep.log; exit 1; }
    echo "resnet w1=$w rep=$rep $(tail -1 $O/resnet_w1${w}_r$rep.log | cut -c1-110)"
  done
done
