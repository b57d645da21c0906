#!/usr/bin/env bash
# round 3 step 42: final tree after the import cleanup -- GPU tier, smoke, bench
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s42_tier 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu || exit 1
run r3_s42_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run r3_s42_bench1 400 python -u bench.py --steps 20 --warmup 5 || exit 1
