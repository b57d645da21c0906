#!/usr/bin/env bash
# round 3 step 34: LDS epilogue on every NT mode (RoPE too): bitwise check; 7B A/B of the fused MLP forward and the
# fused QKV + RoPE projection on top of it
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s34_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_nt_gpu.py || exit 1
for rep in 1 2; do
  DPH_FUSED_MLP=bwd DPH_FUSED_QKV=0 run r3_s34_bench_bwd_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_MLP=1 DPH_FUSED_QKV=0 run r3_s34_bench_mlp_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_MLP=1 DPH_FUSED_QKV=1 run r3_s34_bench_mlpqkv_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
done
run r3_s34_ntbench_all 600 python -u benchmarks/gemm_nt_bench.py --variants 1 --rounds 3 || exit 1
grep -h "TF\|SwiGLU" $O/r3_s34_ntbench_all.log
