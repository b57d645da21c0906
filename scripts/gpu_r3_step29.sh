#!/usr/bin/env bash
# round 3 step 29: in-step A/B of the fused QKV + RoPE projection with the lookahead NT variant (now the default)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
for rep in 1 2; do
  DPH_FUSED_QKV=0 run r3_s29_base_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_QKV=1 run r3_s29_qkv_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
done
