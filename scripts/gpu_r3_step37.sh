#!/usr/bin/env bash
# round 3 step 37: software-pipelined attention forward (DPH_ATTN_FWD_VAR=1) -- bitwise vs attn_fwd_k, kernel A/B,
# interleaved 7B bench A/B
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s37_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "flash or attention" || exit 1
for i in 1 2; do
  run r3_s37_attn_v0_$i 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd || exit 1
  DPH_ATTN_FWD_VAR=1 run r3_s37_attn_v1_$i 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd || exit 1
done
DPH_ATTN_FWD_VAR=1 run r3_s37_attn_v1_nc 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd --noncausal || exit 1
run r3_s37_attn_v0_nc 200 python -u benchmarks/probes/attn_one.py --iters 20 --which fwd --noncausal || exit 1
for i in 1 2; do
  DPH_ATTN_FWD_VAR=1 run r3_s37_bench_v1_$i 400 python -u bench.py --steps 20 --warmup 5 || exit 1
  run r3_s37_bench_v0_$i 400 python -u bench.py --steps 20 --warmup 5 || exit 1
done
