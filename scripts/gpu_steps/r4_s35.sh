#!/bin/bash
# round 4 step 35: SimpleUNet with the c3w_k defaults -- interleaved vs the 1x1 register-staged ts_tn_k (DPH_W1_KERNEL=0)
# and vs MIOpen's 3x3 weight gradient (DPH_CONV3_WGRAD=miopen); step 34's UNet runs were noisy (stdev 0.5-0.7 ms)
set -o pipefail
O=gpurun_out/r4s35; mkdir -p $O
for rep in 1 2; do
  for v in d w m; do
    case $v in d) E="DPH_NOTHING=1";; w) E="DPH_W1_KERNEL=0";; m) E="DPH_CONV3_WGRAD=miopen";; esac
    env $E timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_${v}_r$rep.log 2>&1 || { tail -20 $O/unet_${v}_r$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][0]); print(sys.argv[2], sys.argv[3], d['value'], d['step_ms']['median'], d['step_ms']['stdev'])" $O/unet_${v}_r$rep.log $v $rep
  done
done
bash scripts/prof_bench.sh $O/prof_unet --layout unet-ddp 2>&1 | tail -25
