#!/bin/bash
# round 4 step 40: AdamW with non-temporal loads / stores (DPH_ADAMW_VAR=1) -- bitwise check vs the default, HBM rate
# at 2^28 parameters, 7B in-step A/B interleaved
set -o pipefail
O=gpurun_out/r4s40; mkdir -p $O
cat > $O/adamw_check.py <<'PY'
import os, sys, json, torch
sys.path.insert(0, os.getcwd())
from distributed_pytorch_hpc_amd.ops import _lib
_lib.require()
o = _lib.ops()
n = (1 << 26) + 3
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.randn(n, device="cuda", generator=g); m = torch.randn(n, device="cuda", generator=g).abs() * 1e-3
v = torch.rand(n, device="cuda", generator=g) * 1e-4; gr = torch.randn(n, device="cuda", generator=g).to(torch.bfloat16)
pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    o.adamw_step_(p, m, v, gr, pb, 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.5, None)
torch.cuda.synchronize()
out = sys.argv[1]
torch.save({"p": p.cpu(), "m": m.cpu(), "v": v.cpu(), "pb": pb.cpu()}, out)
PY
DPH_ADAMW_VAR=0 timeout -k 10 120 python -u $O/adamw_check.py $O/a0.pt > $O/chk0.log 2>&1 || { tail -20 $O/chk0.log; exit 1; }
DPH_ADAMW_VAR=1 timeout -k 10 120 python -u $O/adamw_check.py $O/a1.pt > $O/chk1.log 2>&1 || { tail -20 $O/chk1.log; exit 1; }
python3 -c "
import torch
a, b = torch.load('$O/a0.pt', weights_only=True), torch.load('$O/a1.pt', weights_only=True)
print('adamw nt bitwise equal:', all(torch.equal(a[k], b[k]) for k in a))"
rm -f $O/a0.pt $O/a1.pt
for rep in 1 2; do
  for var in 0 1; do
    DPH_ADAMW_VAR=$var timeout -k 10 200 python -u benchmarks/membound_bench.py > $O/mb_var${var}_r$rep.log 2>&1 || { tail -20 $O/mb_var${var}_r$rep.log; exit 1; }
    echo "membound var=$var rep=$rep $(grep -o '"adamw": [0-9.]*' $O/mb_var${var}_r$rep.log)"
  done
done
for rep in 1 2; do
  for var in 0 1; do
    DPH_ADAMW_VAR=$var timeout -k 10 400 python -u bench.py > $O/bench_var${var}_r$rep.log 2>&1 || { tail -20 $O/bench_var${var}_r$rep.log; exit 1; }
    echo "7b var=$var rep=$rep $(grep -o '"value": [0-9.]*' $O/bench_var${var}_r$rep.log)"
  done
done
