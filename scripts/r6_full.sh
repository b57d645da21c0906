#!/bin/bash
# round-6 full validation: the whole GPU test tier, smoke(), and the 1-GPU Llama-2-7B bench
set -o pipefail
out=gpurun_out/r6full
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $out/tier.log 2>&1 || { echo "tier failed"; tail -40 $out/tier.log; exit 1; }
tail -3 $out/tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-500
