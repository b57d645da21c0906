#!/usr/bin/env bash
# round 3 step 28: small-op origins of the ResNet-50, SimpleUNet and Llama-2-7B steps
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u benchmarks/probes/op_origins.py --layout resnet-fsdp --steps 2 > $O/r3_s28_ops_resnet.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/probes/op_origins.py --layout unet-ddp --steps 4 > $O/r3_s28_ops_unet.log 2>&1 || exit 1
timeout -k 10 400 python -u benchmarks/probes/op_origins.py --layout dp --steps 1 > $O/r3_s28_ops_7b.log 2>&1 || exit 1
