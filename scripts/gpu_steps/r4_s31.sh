#!/bin/bash
# round 4 step 31: c3w_k DMA addresses from incrementally advanced pixel coordinates (no per-piece divisions) --
# numerics (1x1 / 3x3 / strided / stem ring variants + strided / stem / UNet tests), per-shape wgrad vs MIOpen
set -o pipefail
O=gpurun_out/r4s31; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_strided_conv_gpu.py -k "conv1x1_wgrad_variants or conv3x3_wgrad_ring_variants or strided or stem or conv3 or unet" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for ns in 2 4; do
  DPH_W1_KERNEL=1 DPH_W1_STAGES=$ns timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --miopen --json $O/w1_ns$ns.json > $O/w1_ns$ns.log 2>&1 || { tail -20 $O/w1_ns$ns.log; exit 1; }
  echo "w1 stages=$ns $(tail -1 $O/w1_ns$ns.log)"
  DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/conv3x3_bench.py --json $O/c3_ns$ns.json > $O/c3_ns$ns.log 2>&1 || { tail -20 $O/c3_ns$ns.log; exit 1; }
  DPH_W1_KERNEL=1 DPH_W1_STAGES=$ns DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/strided_conv_bench.py --json $O/str_ns$ns.json > $O/str_ns$ns.log 2>&1 || { tail -20 $O/str_ns$ns.log; exit 1; }
  echo "strided stages=$ns"; cat $O/str_ns$ns.log | grep -v amdgpu.ids
done
python - <<'PY'
import json
O = "gpurun_out/r4s31"
c = {ns: json.load(open(f"{O}/c3_ns{ns}.json")) for ns in (2, 4)}
print("3x3 wgrad ms".ljust(24) + "miopen".rjust(8) + "".join(f"ns{ns}".rjust(8) for ns in c))
for i, r in enumerate(c[2]["shapes"]):
    print(r["shape"].ljust(24) + f"{r['miopen_wgrad_ms']:8.3f}" + "".join(f"{c[ns]['shapes'][i]['dph_wgrad_ms']:8.3f}" for ns in c))
PY
DPH_C3W_STAGES=2 timeout -k 10 200 python -u benchmarks/stem_conv_bench.py > $O/stem.log 2>&1 || { tail -20 $O/stem.log; exit 1; }
tail -1 $O/stem.log
