#!/bin/bash
# round 4 step 11: strided convolutions per pass vs MIOpen; where the eager SimpleUNet step spends its host time
set -o pipefail
O=gpurun_out/r4s11; mkdir -p $O
timeout -k 10 300 python -u benchmarks/strided_conv_bench.py --json $O/strided.json > $O/strided.log 2>&1 || { tail -30 $O/strided.log; exit 1; }
grep -v amdgpu $O/strided.log
timeout -k 10 300 python -u benchmarks/probes/host_overhead.py --layout unet-ddp --steps 20 --warmup 5 --cprofile 5 --top 60 \
  > $O/unet_host.log 2>&1 || { tail -30 $O/unet_host.log; exit 1; }
grep "\[host\]" $O/unet_host.log
