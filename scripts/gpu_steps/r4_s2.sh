#!/bin/bash
# round 4 step 2: TP fused paths test, TP-rank / PP-stage / UNet benches, wgrad A/B + PMC
set -o pipefail
mkdir -p gpurun_out/r4s2
O=gpurun_out/r4s2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dist_engine_gpu.py \
  > $O/tests_dist_engine.log 2>&1 || { tail -40 $O/tests_dist_engine.log; exit 1; }
tail -2 $O/tests_dist_engine.log
timeout -k 10 300 python -u benchmarks/gemm_nt_bench.py --variants 1 --rounds 3 --no-fused \
  --shapes wqkv.tp8,w13.tp8,w2.tp8,output.tp8,w13.dgrad.tp8,w2.dgrad.tp8,wo.dgrad.tp8 > $O/ntbench_tp8.log 2>&1 || exit 1
grep -v amdgpu.ids $O/ntbench_tp8.log
for nt in fused all; do
  timeout -k 10 300 python -u benchmarks/tp_rank_bench.py --gemm-nt $nt --steps 4 > $O/tp_rank_$nt.log 2>&1 || { tail -20 $O/tp_rank_$nt.log; exit 1; }
  tail -1 $O/tp_rank_$nt.log
done
timeout -k 10 300 python -u benchmarks/pp_stage_bench.py --json $O/pp_stage_v1.json > $O/pp_stage_v1.log 2>&1 || { tail -20 $O/pp_stage_v1.log; exit 1; }
tail -1 $O/pp_stage_v1.log
timeout -k 10 300 python -u benchmarks/pp_stage_bench.py --virtual-stages 2 --json $O/pp_stage_v2.json > $O/pp_stage_v2.log 2>&1 || exit 1
tail -1 $O/pp_stage_v2.log
for prec in bf16 bf16-autocast; do
  timeout -k 10 300 python -u bench.py --layout unet-ddp --unet-precision $prec --steps 30 --warmup 5 > $O/unet_$prec.log 2>&1 || { tail -20 $O/unet_$prec.log; exit 1; }
  tail -1 $O/unet_$prec.log
done
timeout -k 10 300 python -u benchmarks/gemm_mfma_ab.py --variants 32 --rounds 3 > $O/wgrad_ab.log 2>&1 || exit 1
grep -v amdgpu.ids $O/wgrad_ab.log | tail -12
for which in dph blaslt; do
  flag=""; [ $which = blaslt ] && flag=--hipblaslt
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -d /tmp/pmc_$which -o p -- python benchmarks/probes/gemm_one.py $flag > $O/pmc_$which.run.log 2>&1 || exit 1
  db=$(find /tmp/pmc_$which -name "*results.db" -print -quit)
  python benchmarks/pmc_summary.py "$db" > $O/pmc_wgrad_w13_$which.txt 2>&1
  cat $O/pmc_wgrad_w13_$which.txt | head -30
done
