#!/bin/bash
# round 4 step 27: 3x3 / strided / stem weight gradients with deeper c3w_k LDS rings (DPH_C3W_STAGES) -- numerics,
# per-shape wgrad vs MIOpen for each depth
set -o pipefail
O=gpurun_out/r4s27; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "conv3x3_wgrad_ring_variants" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for ns in 2 3 4 5; do
  DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/conv3x3_bench.py --json $O/c3_ns$ns.json > $O/c3_ns$ns.log 2>&1 || { tail -20 $O/c3_ns$ns.log; exit 1; }
  DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/strided_conv_bench.py --json $O/str_ns$ns.json > $O/str_ns$ns.log 2>&1 || { tail -20 $O/str_ns$ns.log; exit 1; }
  echo "stages=$ns"; tail -1 $O/str_ns$ns.log
done
python - <<'PY'
import json
O = "gpurun_out/r4s27"
runs = {ns: json.load(open(f"{O}/c3_ns{ns}.json")) for ns in (2, 3, 4, 5)}
print("3x3 wgrad ms".ljust(24) + "miopen".rjust(8) + "".join(f"ns{ns}".rjust(8) for ns in runs))
for i, r in enumerate(runs[2]["shapes"]):
    print(r["shape"].ljust(24) + f"{r['miopen_wgrad_ms']:8.3f}" + "".join(f"{runs[ns]['shapes'][i]['dph_wgrad_ms']:8.3f}" for ns in runs))
PY
for ns in 2 4; do
  DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/stem_conv_bench.py > $O/stem_ns$ns.log 2>&1 || { tail -20 $O/stem_ns$ns.log; exit 1; }
  echo "stem stages=$ns"; tail -3 $O/stem_ns$ns.log
done
