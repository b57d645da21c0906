#!/bin/bash
# round 6, last tree (after the SimpleUNet decoder / skip folds): the whole GPU tier, smoke(), the 1-GPU Llama-2-7B
# bench, the ResNet-50 FSDP and SimpleUNet benches, and the SimpleUNet kernel profile
set -o pipefail
out=gpurun_out/r6final3
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $out/tier.log 2>&1 || { echo "tier failed"; grep -E "FAILED|Error" $out/tier.log | head; tail -40 $out/tier.log; exit 1; }
tail -1 $out/tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
tail -1 $out/bench_default.log | cut -c1-400
timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/resnet.log 2>&1 || exit 1
tail -1 $out/resnet.log | cut -c1-200
timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 60 --warmup 10 > $out/unet.log 2>&1 || exit 1
tail -1 $out/unet.log | cut -c1-200
timeout -k 10 650 bash scripts/prof_unet.sh $out/unet_prof 20 10 > $out/unet_prof.log 2>&1 || { tail -20 $out/unet_prof.log; exit 1; }
head -12 $out/unet_prof/summary.txt
