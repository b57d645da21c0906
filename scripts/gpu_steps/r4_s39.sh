#!/bin/bash
# round 4 step 39: register-staged weight-gradient kernel (ts_tn_k, the BatchNorm-prologue 1x1 form) split model at its
# real residency (81 VGPRs, 32 KiB LDS: 5 workgroups per CU = 1280) vs the 1024 it assumed -- per shape, ResNet-50 A/B
set -o pipefail
O=gpurun_out/r4s39; mkdir -p $O
for R in 1024 1280; do
  DPH_W1_KERNEL=0 DPH_TS_TN_WGS=$R timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/ts_R$R.json > $O/ts_R$R.log 2>&1 || { tail -20 $O/ts_R$R.log; exit 1; }
  echo "R=$R $(tail -1 $O/ts_R$R.log)"
done
python3 - <<'PY'
import json
O = "gpurun_out/r4s39"
a, b = json.load(open(f"{O}/ts_R1024.json")), json.load(open(f"{O}/ts_R1280.json"))
for x, y in zip(a["rows"], b["rows"]):
    print(f"{x['cin']:5d}->{x['cout']:5d} @{x['H']:3d} x{x['count']}  R1024 {x['ms']:.3f}  R1280 {y['ms']:.3f}  {x['ms'] / y['ms']:.2f}x")
PY
for rep in 1 2; do
  for R in 1024 1280; do
    DPH_TS_TN_WGS=$R timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_R${R}_r$rep.log 2>&1 || { tail -20 $O/resnet_R${R}_r$rep.log; exit 1; }
    echo "resnet R=$R rep=$rep $(grep '^{"metric' $O/resnet_R${R}_r$rep.log | cut -c60-130)"
  done
done
