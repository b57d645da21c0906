#!/bin/bash
# round 4 step 30: c3w_k with identity rows for the 1x1 weight gradient (GEN 3) and the next DMA issued behind the
# first k-step's LDS reads -- numerics, 1x1 and 3x3 sweeps at ring depth 2 / 4
set -o pipefail
O=gpurun_out/r4s30; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "conv1x1_wgrad_variants or conv3x3_wgrad_ring_variants" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
DPH_W1_KERNEL=0 timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_ts.json > $O/w1_ts.log 2>&1 || { tail -20 $O/w1_ts.log; exit 1; }
tail -1 $O/w1_ts.log
for ns in 2 4; do
  DPH_W1_KERNEL=1 DPH_W1_STAGES=$ns timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_ns$ns.json > $O/w1_ns$ns.log 2>&1 || { tail -20 $O/w1_ns$ns.log; exit 1; }
  echo "w1 stages=$ns $(tail -1 $O/w1_ns$ns.log)"
  DPH_C3W_STAGES=$ns timeout -k 10 200 python -u benchmarks/conv3x3_bench.py --json $O/c3_ns$ns.json > $O/c3_ns$ns.log 2>&1 || { tail -20 $O/c3_ns$ns.log; exit 1; }
done
python - <<'PY'
import json
O = "gpurun_out/r4s30"
runs = {"ts": json.load(open(f"{O}/w1_ts.json")), "ns2": json.load(open(f"{O}/w1_ns2.json")), "ns4": json.load(open(f"{O}/w1_ns4.json"))}
print("1x1 wgrad".ljust(22) + "".join(k.rjust(8) for k in runs))
for i, r in enumerate(runs["ts"]["rows"]):
    print(f"{r['cin']:5d}->{r['cout']:5d} @{r['H']:3d} x{r['count']}".ljust(22) + "".join(f"{runs[k]['rows'][i]['ms']:8.3f}" for k in runs))
c = {ns: json.load(open(f"{O}/c3_ns{ns}.json")) for ns in (2, 4)}
print("3x3 wgrad ms".ljust(24) + "miopen".rjust(8) + "".join(f"ns{ns}".rjust(8) for ns in c))
for i, r in enumerate(c[2]["shapes"]):
    print(r["shape"].ljust(24) + f"{r['miopen_wgrad_ms']:8.3f}" + "".join(f"{c[ns]['shapes'][i]['dph_wgrad_ms']:8.3f}" for ns in c))
PY
