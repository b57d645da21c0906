#!/usr/bin/env bash
# round 3 step 24: world-1 ZeRO-3 with unit buffers aliased to the shards (no gather / scatter copies): ResNet-50 A/B
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s24_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "resnet or fsdp or graph or bench" || exit 1
for rep in 1 2; do for a in 0 1; do
  DPH_FSDP_ALIAS=$a run r3_s24_resnet_a${a}_rep$rep 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
done; done
DPH_FSDP_ALIAS=1 run r3_s24_unet 400 python -u bench.py --layout unet-ddp --steps 100 --warmup 10 || exit 1
