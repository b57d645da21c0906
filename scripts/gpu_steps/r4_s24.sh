#!/bin/bash
# round 4 step 24: SimpleUNet eager vs whole-step HIP graph after the launch cuts (interleaved), graph-mode profile
set -o pipefail
O=gpurun_out/r4s24; mkdir -p $O
for rep in 1 2; do
  for g in 0 1; do
    flag=""; [ $g = 1 ] && flag=--graph
    timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 $flag > $O/unet_graph${g}_r$rep.log 2>&1 || { tail -20 $O/unet_graph${g}_r$rep.log; exit 1; }
    echo "unet graph=$g rep=$rep $(grep '^{"metric' $O/unet_graph${g}_r$rep.log | cut -c1-110)"
  done
done
bash scripts/prof_bench.sh $O/prof_unet_graph --layout unet-ddp --graph 2>&1 | tail -30
