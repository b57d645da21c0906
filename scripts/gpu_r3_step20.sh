#!/usr/bin/env bash
# round 3 step 20: NT GEMM 2-phase variant (32 MFMAs per barrier segment): parity + A/B vs hipBLASLt
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s20_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py || exit 1
run r3_s20_bench 600 python -u benchmarks/gemm_nt_bench.py --variants 0,1,2 --rounds 3 --json $O/r3_s20_gemm_nt_bench.json || exit 1
