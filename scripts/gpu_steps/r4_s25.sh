#!/bin/bash
# round 4 step 25: 1x1 weight gradient with a deeper LDS-DMA ring (DPH_W1_STAGES) -- numerics, per-shape sweep vs ts_tn_k
set -o pipefail
O=gpurun_out/r4s25; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "conv1x1_wgrad_variants" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
DPH_W1_KERNEL=0 timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_ts.json > $O/w1_ts.log 2>&1 || { tail -20 $O/w1_ts.log; exit 1; }
tail -1 $O/w1_ts.log
for ns in 2 3 4 5; do
  DPH_W1_KERNEL=1 DPH_W1_STAGES=$ns timeout -k 10 120 python -u benchmarks/conv1x1_wgrad_bench.py --json $O/w1_ns$ns.json > $O/w1_ns$ns.log 2>&1 || { tail -20 $O/w1_ns$ns.log; exit 1; }
  echo "stages=$ns $(tail -1 $O/w1_ns$ns.log)"
done
python - <<'PY'
import json
O = "gpurun_out/r4s25"
runs = {"ts": json.load(open(f"{O}/w1_ts.json"))}
for ns in (2, 3, 4, 5):
    runs[f"ns{ns}"] = json.load(open(f"{O}/w1_ns{ns}.json"))
keys = list(runs)
print("shape".ljust(22) + "".join(k.rjust(8) for k in keys))
for i, r in enumerate(runs["ts"]["rows"]):
    print(f"{r['cin']:5d}->{r['cout']:5d} @{r['H']:3d} x{r['count']}".ljust(22) + "".join(f"{runs[k]['rows'][i]['ms']:8.3f}" for k in keys))
PY
