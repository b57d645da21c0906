#!/usr/bin/env bash
# round 3 step 33: NT GEMM epilogue through LDS (STORE / SWIGLU / DSWIGLU): bitwise check, per-GEMM bench, 7B A/B
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s33_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_nt_gpu.py || exit 1
for form in reg lds; do
  DPH_NT_EPI=$form run r3_s33_ntbench_$form 400 python -u benchmarks/gemm_nt_bench.py --variants 1 --rounds 3 --shapes wqkv,w13,w2.dgrad,output || exit 1
  grep -h "TF\|SwiGLU" $O/r3_s33_ntbench_$form.log
done
for rep in 1 2; do
  DPH_NT_EPI=reg run r3_s33_bench_reg_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  run r3_s33_bench_lds_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_MLP=1 run r3_s33_bench_ldsfwd_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
done
