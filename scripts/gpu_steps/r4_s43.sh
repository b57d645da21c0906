#!/bin/bash
# round 4 step 43: bn2's apply as its own pass (DPH_BN_PROLOGUE=0) now that the plain 1x1 weight gradient runs on the
# faster c3w_k identity-row kernel (the prologue form keeps conv3's weight gradient on ts_tn_k) -- ResNet-50 A/B
set -o pipefail
O=gpurun_out/r4s43; mkdir -p $O
for rep in 1 2 3; do
  for v in 1 0; do
    DPH_BN_PROLOGUE=$v timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_pro${v}_r$rep.log 2>&1 || { tail -20 $O/resnet_pro${v}_r$rep.log; exit 1; }
    echo "resnet prologue=$v rep=$rep $(grep -o '"value": [0-9.]*' $O/resnet_pro${v}_r$rep.log)"
  done
done
