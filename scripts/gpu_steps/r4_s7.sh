#!/bin/bash
# round 4 step 7: NT GEMM vs hipBLASLt PMC (wqkv shape), UNet 3x3 wgrad dph vs MIOpen
set -o pipefail
O=gpurun_out/r4s7; mkdir -p $O
export TMPDIR=/tmp
for which in dph blaslt; do
  flag=""; [ $which = blaslt ] && flag=--hipblaslt
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -d /tmp/pmcnt_$which -o p -- python benchmarks/probes/nt_one.py $flag > $O/pmc_$which.run.log 2>&1 || exit 1
  db=$(find /tmp/pmcnt_$which -name "*results.db" -print -quit)
  python benchmarks/pmc_summary.py "$db" > $O/pmc_nt_wqkv_$which.txt 2>&1
  grep -B1 -A20 "gemm_nt\|Cijk" $O/pmc_nt_wqkv_$which.txt | grep -E "==|dur|dispatch|mfma_busy|clock|WAIT|vgpr|agpr|LDS|WAVE_CYCLES"
done
for rep in 1 2; do
  for wg in miopen dph; do
    DPH_CONV3_WGRAD=$wg timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 > $O/unet_wg_${wg}_r$rep.log 2>&1 || { tail -20 $O/unet_wg_${wg}_r$rep.log; exit 1; }
    echo "$wg rep=$rep $(tail -1 $O/unet_wg_${wg}_r$rep.log | cut -c1-120)"
  done
done
