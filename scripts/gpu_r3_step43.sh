#!/usr/bin/env bash
# round 3 step 43: Llama-2-13B training on ONE MI355X (fp32 master + AdamW state resident: ~208 GB static)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"peak_hbm_gb": [0-9.]*' $O/$name.log | tr '\n' ' ')"; return $rc; }
run r3_s43_13b_b2 500 python -u bench.py --model llama2-13b --micro-batch 2 --steps 6 --warmup 2 || exit 1
run r3_s43_13b_b4_ac 600 python -u bench.py --model llama2-13b --micro-batch 4 --ac auto --steps 6 --warmup 2 || exit 1
