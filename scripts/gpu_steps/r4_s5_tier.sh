#!/bin/bash
# round 4 step 5: the full GPU test tier + smoke on the current tree
set -o pipefail
O=gpurun_out/r4s5; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1
rc=$?
tail -15 $O/gpu_tier.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
