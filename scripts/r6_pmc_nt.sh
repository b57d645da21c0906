#!/bin/bash
# round-6: PMC pass of the projection GEMM forms on the wqkv shape: hipBLASLt, gemm_nt_k (8 waves), gemm_nt4_k (4 waves)
set -o pipefail
out=gpurun_out/r6/nt4_pmc
mkdir -p $out
export TMPDIR=/tmp
ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for arm in blaslt nt8 nt4; do
  case $arm in blaslt) extra="--hipblaslt";; nt8) extra="--variant 0";; nt4) extra="--variant 6";; esac
  raw=/tmp/pmc_$arm; rm -rf $raw
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $raw -o p -- python3 benchmarks/probes/nt_one.py --iters 6 $extra > $out/run_$arm.log 2>&1 || exit 1
  db=$(find $raw -name "*results.db" -print -quit)
  python3 benchmarks/pmc_summary.py "$db" --match "Cijk|gemm_nt" > $out/pmc_$arm.txt || exit 1
  echo "== $arm"; cat $out/pmc_$arm.txt
done
