#!/bin/bash
# round 4 step 17: one TP = 8 rank's 7B compute with the ragged 16x16x32 NT kernel: hipBLASLt only vs fused MLP (default)
# vs every projection on the NT kernel, and the fused QKV + RoPE path
set -o pipefail
O=gpurun_out/r4s17; mkdir -p $O
for rep in 1 2; do
  for nt in 0 fused all; do
    timeout -k 10 300 python -u benchmarks/tp_rank_bench.py --gemm-nt $nt --steps 4 > $O/tp_rank_${nt}_r$rep.log 2>&1 || { tail -20 $O/tp_rank_${nt}_r$rep.log; exit 1; }
    echo "nt=$nt rep=$rep $(tail -1 $O/tp_rank_${nt}_r$rep.log)"
  done
  timeout -k 10 300 python -u benchmarks/tp_rank_bench.py --gemm-nt all --fused-qkv 1 --steps 4 > $O/tp_rank_allqkv_r$rep.log 2>&1 || { tail -20 $O/tp_rank_allqkv_r$rep.log; exit 1; }
  echo "nt=all+qkv rep=$rep $(tail -1 $O/tp_rank_allqkv_r$rep.log)"
done
# the 7B step with the dQ kernel variants, interleaved (default 2 = spill-free quarter read-ahead)
for rep in 1 2; do
  for v in 0 2; do
    DPH_ATTN_DQ_VAR=$v timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 > $O/bench_dq${v}_r$rep.log 2>&1 || { tail -20 $O/bench_dq${v}_r$rep.log; exit 1; }
    echo "7b dq=$v rep=$rep $(tail -1 $O/bench_dq${v}_r$rep.log | cut -c1-120)"
  done
done
