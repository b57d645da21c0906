#!/usr/bin/env bash
# round 3 step 13: full GPU tier with the 3x3 path on by default, then the bench layouts (headline, ResNet-50, UNet)
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 600 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s13_gpu_tier python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/
rc=$?; [ $rc -le 1 ] || exit $rc
run r3_s13_bench_dp python -u bench.py --steps 6 --warmup 2 --json-out $O/r3_s13_bench_dp.json || exit 1
run r3_s13_resnet python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --json-out $O/r3_s13_resnet.json || exit 1
run r3_s13_resnet_graph python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --graph --json-out $O/r3_s13_resnet_graph.json || exit 1
run r3_s13_unet python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_s13_unet.json || exit 1
run r3_s13_unet_graph python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --graph --json-out $O/r3_s13_unet_graph.json || exit 1
