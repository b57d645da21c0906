#!/usr/bin/env bash
# round 3 step 23: in-step A/B of the backward-only fused MLP (dSwiGLU in w2's input-gradient epilogue) with the
# lookahead NT GEMM variant, against the library path; interleaved, two reps
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s23_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py || exit 1
for rep in 1 2; do
  DPH_FUSED_MLP=0 run r3_s23_base_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_MLP=bwd DPH_GEMM_NT_VARIANT=1 run r3_s23_bwdv1_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
  DPH_FUSED_MLP=bwd DPH_GEMM_NT_VARIANT=0 run r3_s23_bwdv0_rep$rep 400 python -u bench.py --steps 10 --warmup 3 || exit 1
done
run r3_s23_resnet 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
timeout -k 10 500 bash scripts/prof_resnet.sh $O/r3_s23_prof_resnet 256 10 > $O/r3_s23_prof_resnet.log 2>&1; echo "prof_resnet rc=$?"
