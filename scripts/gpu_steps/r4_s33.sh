#!/bin/bash
# round 4 step 33: c3w_k split-K chunks filling exactly one resident round (floor instead of ceil) -- numerics and
# per-shape 1x1 / 3x3 / strided / stem weight gradients vs MIOpen
set -o pipefail
O=gpurun_out/r4s33; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_strided_conv_gpu.py -k "conv1x1_wgrad_variants or conv3x3_wgrad_ring_variants or strided or stem or conv3 or unet" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
DPH_W1_KERNEL=1 timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --miopen --json $O/w1.json > $O/w1.log 2>&1 || { tail -20 $O/w1.log; exit 1; }
grep -v amdgpu.ids $O/w1.log
timeout -k 10 200 python -u benchmarks/conv3x3_bench.py --json $O/c3.json > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
python - <<'PY'
import json
c = json.load(open("gpurun_out/r4s33/c3.json"))
for r in c["shapes"]:
    print(f"{r['shape']:24s} wgrad miopen {r['miopen_wgrad_ms']:.3f} dph {r['dph_wgrad_ms']:.3f} ({r['miopen_wgrad_ms'] / r['dph_wgrad_ms']:.2f}x)")
PY
DPH_W1_KERNEL=1 timeout -k 10 200 python -u benchmarks/strided_conv_bench.py --json $O/str.json > $O/str.log 2>&1 || { tail -20 $O/str.log; exit 1; }
grep -v amdgpu.ids $O/str.log
timeout -k 10 200 python -u benchmarks/stem_conv_bench.py > $O/stem.log 2>&1 || { tail -20 $O/stem.log; exit 1; }
tail -1 $O/stem.log
