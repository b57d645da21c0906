#!/bin/bash
# round 4 step 6: staggered 8-wave attention forward (numerics + A/B vs 4 / 8 waves), UNet precision A/B (alternating)
set -o pipefail
O=gpurun_out/r4s6; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "eight_wave" \
  > $O/tests_attn.log 2>&1 || { tail -30 $O/tests_attn.log; exit 1; }
tail -2 $O/tests_attn.log
for rep in 1 2; do
  for w in 4 8 9; do
    DPH_ATTN_WAVES=$w timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which fwd --iters 20 > $O/attn_w${w}_r$rep.log 2>&1 || { tail $O/attn_w${w}_r$rep.log; exit 1; }
    echo "w=$w rep=$rep $(grep -v amdgpu $O/attn_w${w}_r$rep.log | tail -1)"
  done
done
for rep in 1 2; do
  for prec in bf16 bf16-autocast; do
    timeout -k 10 300 python -u bench.py --layout unet-ddp --unet-precision $prec --steps 40 --warmup 8 > $O/unet_${prec}_r$rep.log 2>&1 || { tail -20 $O/unet_${prec}_r$rep.log; exit 1; }
    echo "$prec rep=$rep $(tail -1 $O/unet_${prec}_r$rep.log | cut -c1-120)"
  done
done
