#!/bin/bash
# round 4 step 16: is the ResNet-50 step host-bound now (enqueue vs device time, cProfile)?  UNet stats A/B again.
set -o pipefail
O=gpurun_out/r4s16; mkdir -p $O
timeout -k 10 300 python -u benchmarks/probes/host_overhead.py --layout resnet-fsdp --steps 10 --warmup 3 --cprofile 3 --top 50 \
  > $O/resnet_host.log 2>&1 || { tail -30 $O/resnet_host.log; exit 1; }
grep "\[host\]" $O/resnet_host.log
for rep in 1 2 3; do
  for st in 0 1; do
    DPH_UNET_CONV_STATS=$st timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_stats${st}_r$rep.log 2>&1 || { tail -20 $O/unet_stats${st}_r$rep.log; exit 1; }
    echo "unet stats=$st rep=$rep $(tail -1 $O/unet_stats${st}_r$rep.log | cut -c1-110)"
  done
done
