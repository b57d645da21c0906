#!/bin/bash
# round 4 step 44: the full GPU test tier + smoke + the default bench on the current tree
set -o pipefail
O=gpurun_out/r4s44; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1
rc=$?
tail -15 $O/gpu_tier.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet.log 2>&1 || { tail -20 $O/resnet.log; exit 1; }
grep "^{\"metric" $O/resnet.log | cut -c1-160
