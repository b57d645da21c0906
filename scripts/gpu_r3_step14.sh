#!/usr/bin/env bash
# round 3 step 14: RCCL with two ranks on one GPU (probe), whole-step graphs for the UNet / ResNet layouts
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s14_rccl_shared python -u scripts/probe_rccl_shared_gpu.py
run r3_s14_unet python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_s14_unet.json || exit 1
run r3_s14_unet_graph python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --graph --json-out $O/r3_s14_unet_graph.json || exit 1
run r3_s14_resnet_graph python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --graph --json-out $O/r3_s14_resnet_graph.json
