#!/usr/bin/env bash
# round 3 step 15: in-step A/B of the fused QKV+RoPE projection and of the dK/dV read pipelining (Llama-2-7B bench)
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log)"; return $rc; }
for rep in 1 2; do
  run r3_s15_base_rep$rep python -u bench.py --steps 6 --warmup 2 || exit 1
  DPH_FUSED_QKV=1 run r3_s15_qkv_rep$rep python -u bench.py --steps 6 --warmup 2 || exit 1
  DPH_ATTN_BWD_VAR=0 run r3_s15_dkdv0_rep$rep python -u bench.py --steps 6 --warmup 2 || exit 1
done
