#!/usr/bin/env bash
# round 3 step 17: BatchNorm-apply + ReLU folded into the 1x1 convolution (parity, ResNet-50 A/B)
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log)"; return $rc; }
run r3_s17_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prologue or bottleneck or resnet or conv1x1 or tall_skinny" || exit 1
run r3_s17_resnet_tests python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "resnet" || exit 1
for rep in 1 2; do for p in 0 1; do
  DPH_BN_PROLOGUE=$p run r3_s17_resnet_p${p}_rep$rep python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --json-out $O/r3_s17_resnet_p${p}_rep$rep.json || exit 1
done; done
