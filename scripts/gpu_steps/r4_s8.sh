#!/bin/bash
# round 4 step 8: ragged edge tiles on the 16x16x32 NT kernel (numerics for all variants), TP8 shard A/B 1 vs 3
set -o pipefail
O=gpurun_out/r4s8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py \
  > $O/tests_nt.log 2>&1 || { tail -30 $O/tests_nt.log; exit 1; }
tail -2 $O/tests_nt.log
timeout -k 10 300 python -u benchmarks/gemm_nt_bench.py --variants 1,3 \
  --shapes wqkv.tp8,w13.tp8,w2.tp8,output.tp8,w13.dgrad.tp8,w2.dgrad.tp8,wo.dgrad.tp8 \
  --json $O/nt_tp8.json > $O/nt_tp8.log 2>&1 || { tail -30 $O/nt_tp8.log; exit 1; }
cat $O/nt_tp8.log | grep -v amdgpu
for rep in 1 2; do
  for wg in miopen dph; do
    DPH_CONV3_WGRAD=$wg timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 > $O/resnet_wg_${wg}_r$rep.log 2>&1 || { tail -20 $O/resnet_wg_${wg}_r$rep.log; exit 1; }
    echo "resnet $wg rep=$rep $(tail -1 $O/resnet_wg_${wg}_r$rep.log | cut -c1-110)"
  done
done
DPH_CONV3_WGRAD=dph bash scripts/prof_bench.sh $O/prof_unet_dph --layout unet-ddp
