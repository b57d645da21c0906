#!/bin/bash
# round 4 step 17: one TP = 8 rank's 7B compute with the ragged 16x16x32 NT kernel: hipBLASLt only vs fused MLP (default)
# vs every projection on the NT kernel; the 7B step with the dQ variants.  Every step prints progress (the previous
# attempt was killed for 180 s of silence while the first process paged torch in and built the model).
set -o pipefail
O=gpurun_out/r4s17; mkdir -p $O
timeout -k 10 200 python -u -c "import torch; print('torch', torch.__version__, torch.cuda.is_available(), flush=True)"
for rep in 1 2; do
  for nt in fused 0 all; do
    timeout -k 10 300 python -u benchmarks/tp_rank_bench.py --gemm-nt $nt --steps 4 2>&1 | tee $O/tp_rank_${nt}_r$rep.log | grep --line-buffered "tp_rank\|ms_per_step" || { tail -20 $O/tp_rank_${nt}_r$rep.log; exit 1; }
  done
done
for rep in 1 2; do
  for v in 0 2; do
    DPH_ATTN_DQ_VAR=$v timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 2>&1 | tee $O/bench_dq${v}_r$rep.log | grep --line-buffered "^{" | cut -c1-120 || { tail -20 $O/bench_dq${v}_r$rep.log; exit 1; }
  done
done
