#!/bin/bash
# round 4 step 41: strided 1x1 weight gradient on the gathered c3w_k tiles (no sub-image copy) -- numerics, per-pass
# bench, ResNet-50 A/B vs the copy path (DPH_STRIDED1_COPY=1), interleaved
set -o pipefail
O=gpurun_out/r4s41; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_strided_conv_gpu.py \
  tests/test_kernels_gpu.py -k "strided or Strided or bottleneck or sub or conv3x3_wgrad_ring or conv1x1_wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u benchmarks/strided_conv_bench.py --json $O/str.json > $O/str.log 2>&1 || { tail -20 $O/str.log; exit 1; }
grep -v amdgpu.ids $O/str.log
for rep in 1 2; do
  for v in 1 0; do
    DPH_STRIDED1_COPY=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_copy${v}_r$rep.log 2>&1 || { tail -20 $O/resnet_copy${v}_r$rep.log; exit 1; }
    echo "resnet copy=$v rep=$rep $(grep -o '"value": [0-9.]*' $O/resnet_copy${v}_r$rep.log)"
  done
done
