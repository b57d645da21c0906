#!/bin/bash
# round 4 step 38: 1x1 forward / input-gradient kernel (ts_nt_k) at 4 workgroups per CU (128 VGPRs) vs 3 -- numerics,
# grid-tail probe per occupancy, ResNet-50 in-step A/B (DPH_TS_NT_OCC=3 = the old build), interleaved
set -o pipefail
O=gpurun_out/r4s38; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_strided_conv_gpu.py -k "conv1x1 or ts_gemm or bottleneck or resnet or strided or sub" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for occ in 4 3; do
  DPH_TS_NT_OCC=$occ timeout -k 10 300 python -u benchmarks/probes/grid_tail.py > $O/grid_tail_occ$occ.log 2>&1 || { tail -20 $O/grid_tail_occ$occ.log; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4s38"
r = {occ: [json.loads(l) for l in open(f"{O}/grid_tail_occ{occ}.log") if l.startswith("{")] for occ in (4, 3)}
for a, b in zip(r[4], r[3]):
    if a["kind"] == "1x1" and a["row_tiles"] in (128, 256, 384, 392, 512, 768, 784):
        print(a["kind"], a["N"], a["K"], a["row_tiles"], "occ4", a["ms"], "occ3", b["ms"], f"{b['ms'] / a['ms']:.2f}x")
PY
for rep in 1 2; do
  for occ in 3 4; do
    DPH_TS_NT_OCC=$occ timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_occ${occ}_r$rep.log 2>&1 || { tail -20 $O/resnet_occ${occ}_r$rep.log; exit 1; }
    echo "resnet occ=$occ rep=$rep $(grep '^{"metric' $O/resnet_occ${occ}_r$rep.log | cut -c60-130)"
  done
done
