#!/bin/bash
# round 6, last tree (after the weight-gradient split knob): the whole GPU tier and smoke()
set -o pipefail
out=gpurun_out/r6final4
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $out/tier.log 2>&1 || { echo "tier failed"; grep -E "FAILED|Error" $out/tier.log | head; tail -40 $out/tier.log; exit 1; }
tail -1 $out/tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
