#!/bin/bash
# round-6: PMC pass over the attention kernels (variant 0 = 16x16x32 forms, 1 = 32x32x16), per-kernel summary
set -o pipefail
out=gpurun_out/${1:-r6_pmc}
mkdir -p $out
export TMPDIR=/tmp
ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-0 1}; do
  raw=/tmp/pmc_v$v
  rm -rf $raw
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $raw -o p -- python3 benchmarks/probes/attn_one.py --iters 4 --variant $v > $out/pmc_run_v$v.log 2>&1 || exit 1
  db=$(find $raw -name "*results.db" -print -quit)
  python3 benchmarks/pmc_summary.py "$db" --match "attn_" --json $out/pmc_v$v.json > $out/pmc_v$v.txt || exit 1
  echo "== variant $v"; cat $out/pmc_v$v.txt
done
