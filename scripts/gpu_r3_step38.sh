#!/usr/bin/env bash
# round 3 step 38: pipelined attention forward, compiler-scheduled form (DPH_ATTN_FWD_VAR=2) and 8-wave workgroups
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s38_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pipelined or eight_wave" || exit 1
for i in 1 2; do
  for v in 0 1 2; do
    DPH_ATTN_FWD_VAR=$v run r3_s38_attn_v${v}_w4_$i 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd || exit 1
    DPH_ATTN_WAVES=8 DPH_ATTN_FWD_VAR=$v run r3_s38_attn_v${v}_w8_$i 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd || exit 1
  done
done
