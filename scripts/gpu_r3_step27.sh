#!/usr/bin/env bash
# round 3 step 27: ResNet-50 small-kernel trims -- BN partial merge sized to the partial count, HIP transposes for
# the input-gradient weights -- parity + interleaved A/B against the previous forms
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s27_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "conv3x3 or bottleneck or resnet or bn or batchnorm or weight_t or unet or conv1x1 or tall_skinny" || exit 1
for rep in 1 2; do
  DPH_BN_MERGE_LEGACY=1 DPH_CONV_WT=aten run r3_s27_resnet_old_rep$rep 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
  run r3_s27_resnet_new_rep$rep 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
done
