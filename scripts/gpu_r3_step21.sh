#!/usr/bin/env bash
# round 3 step 21: attention backward with the dS hand-off (dK/dV kernel writes dS, dQ = dS K only)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
true
for rep in 1 2; do for ds in 0 1; do
  DPH_ATTN_DS=$ds run r3_s21_attn_ds${ds}_rep$rep 300 python -u benchmarks/probes/attn_one.py --which bwd --iters 10 || exit 1
  grep bwd $O/r3_s21_attn_ds${ds}_rep$rep.log
done; done
run r3_s21_prof 300 rocprofv3 --kernel-trace --stats -d $O/r3_s21_prof -o prof -- python -u benchmarks/probes/attn_one.py --which bwd --iters 3 || exit 1
for ds in 1 0; do
  DPH_ATTN_DS=$ds run r3_s21_bench_ds$ds 600 python -u bench.py --steps 10 --warmup 3 || exit 1
done
