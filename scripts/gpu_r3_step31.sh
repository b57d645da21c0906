#!/usr/bin/env bash
# round 3 step 31: BatchNorm-backward statistics from the 1x1 input-gradient epilogues -- parity + ResNet-50 A/B
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s31_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "bnstats or bn_bwd_stats or bottleneck" || exit 1
for rep in 1 2; do
  DPH_BN_BWD_STATS=0 run r3_s31_resnet_off_rep$rep 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
  run r3_s31_resnet_on_rep$rep 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
done
