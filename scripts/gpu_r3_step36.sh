#!/usr/bin/env bash
# round 3 step 36: attention epilogues through LDS -- numerics (attention / RoPE / ring tests), kernel A/B against the
# per-lane row stores (DPH_ATTN_EPI=reg), interleaved 7B bench A/B
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s36_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "flash or attention or attn or ring or rope or decode" || exit 1
for i in 1 2; do
  run r3_s36_attn_lds$i 200 python -u benchmarks/probes/attn_one.py --iters 10 || exit 1
  DPH_ATTN_EPI=reg run r3_s36_attn_reg$i 200 python -u benchmarks/probes/attn_one.py --iters 10 || exit 1
done
for i in 1 2; do
  run r3_s36_bench_lds$i 400 python -u bench.py --steps 20 --warmup 5 || exit 1
  DPH_ATTN_EPI=reg run r3_s36_bench_reg$i 400 python -u bench.py --steps 20 --warmup 5 || exit 1
done
